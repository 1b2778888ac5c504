#!/bin/bash
# r04: config 5 — where the step goes (phases, submit time), kernel trace with list-sized bundles.
set -o pipefail
out=gpurun_out/j19
mkdir -p $out
GCK_DEBUG_PHASES=1 timeout -k 10 300 python -u bench.py --config mixed --steps 20 --warmup 5 > $out/mixed.json 2> $out/mixed.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/kt -o mixed -- python3 -u bench.py --config mixed --steps 20 --warmup 5 --no-cpu > $out/kt_mixed.json 2> $out/kt_mixed.err || exit 2
find $out -type f -size +4M -delete
