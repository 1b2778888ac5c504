#!/bin/bash
# r04 probe: does the Watch batch's merge wait behind the check batch in a shared hardware queue?
set -o pipefail
out=gpurun_out/j36
mkdir -p $out
for q in 4 8 16; do
GPU_MAX_HW_QUEUES=$q GCK_DEBUG_PHASES=1 timeout -k 10 300 python -u bench.py --config mixed --steps 20 --warmup 5 --no-cpu > $out/mixed_q$q.json 2> $out/mixed_q$q.err || exit 2
done
