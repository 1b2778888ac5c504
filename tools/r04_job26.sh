#!/bin/bash
# r04: packing rule (no extra extension records for a narrower slot); configs 2, 3.
set -o pipefail
out=gpurun_out/j27
mkdir -p $out
for cfg in gdocs github; do
  GCK_DEBUG_PHASES=1 timeout -k 10 240 python -u bench.py --config $cfg --steps 200 --warmup 5 > $out/$cfg.json 2> $out/$cfg.err || exit 2
done
