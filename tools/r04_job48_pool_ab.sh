#!/bin/bash
set -o pipefail
out=gpurun_out/j48
mkdir -p $out
for r in 1 2 3; do
GCK_DEBUG_PHASES=1 timeout -k 10 300 python -u bench.py --config mixed --steps 20 --warmup 5 --no-cpu --no-oracle > $out/pool_$r.json 2> $out/pool_$r.err || exit 2
GCK_TMP_SERIAL=1 GCK_DEBUG_PHASES=1 timeout -k 10 300 python -u bench.py --config mixed --steps 20 --warmup 5 --no-cpu --no-oracle > $out/serial_$r.json 2> $out/serial_$r.err || exit 2
done
