#!/bin/bash
# r04: config 5 — the step's parts (apply, submit, wait), phases on and off.
set -o pipefail
out=gpurun_out/j20
mkdir -p $out
timeout -k 10 300 python -u bench.py --config mixed --steps 20 --warmup 5 --no-cpu > $out/mixed.json 2> $out/mixed.err || exit 1
GCK_DEBUG_PHASES=1 timeout -k 10 300 python -u bench.py --config mixed --steps 20 --warmup 5 --no-cpu > $out/mixed_ph.json 2> $out/mixed_ph.err || exit 2
