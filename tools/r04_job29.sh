#!/bin/bash
set -o pipefail
out=gpurun_out/j29
mkdir -p $out
for r in 1 2; do
  timeout -k 10 240 python -u bench.py --no-profile > $out/on_$r.json 2> $out/on_$r.err || exit 3
  GCK_EXP_NOSTAMPS=1 timeout -k 10 240 python -u bench.py --no-profile > $out/off_$r.json 2> $out/off_$r.err || exit 3
done
