#!/bin/bash
set -o pipefail
out=gpurun_out/j24
mkdir -p $out
GCK_DEBUG_PHASES=1 timeout -k 10 300 python -u bench.py --config mixed --steps 20 --warmup 5 --no-cpu > $out/mixed_ph.json 2> $out/mixed_ph.err || exit 3
