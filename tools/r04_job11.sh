#!/bin/bash
# r04: config 5's chained bundles — kernel traces with and without the label stage, and the
# check-stage phase of the bench.
set -o pipefail
out=gpurun_out/j11
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kt_nolabels -o kt --output-format csv -- \
  python3 bench.py --config mixed --steps 20 --warmup 5 --no-cpu --no-labels > $out/kt_nolabels.json 2> $out/kt_nolabels.err || exit 1
timeout -k 10 300 python -u bench.py --config mixed --steps 20 --warmup 5 > $out/mixed.json 2> $out/mixed.err || exit 2
find $out -name "*kernel_trace.csv" -delete
find $out -name "*agent_info.csv" -delete
