#!/bin/bash
# r04 A/B: a short bundle list over half the slots (the rest free for a Watch batch's kernels).
set -o pipefail
out=gpurun_out/j32
mkdir -p $out
for r in 1 2; do
timeout -k 10 300 python -u bench.py --config mixed --steps 20 --warmup 5 --no-cpu > $out/mixed_$r.json 2> $out/mixed_$r.err || exit 2
done
GCK_DEBUG_PHASES=1 timeout -k 10 300 python -u bench.py --config mixed --steps 20 --warmup 5 --no-cpu > $out/mixed_ph.json 2> $out/mixed_ph.err || exit 3
