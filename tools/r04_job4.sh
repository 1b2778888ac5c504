#!/bin/bash
# r04: label join checks per wave A/B on configs 2 and 3 (GCK_LJ_CPW 32 / 16), driver-sized runs.
set -o pipefail
out=gpurun_out/j4
mkdir -p $out
for cfg in gdocs github; do
  for cpw in 32 16; do
    GCK_LJ_CPW=$cpw timeout -k 10 240 python -u bench.py --config $cfg --steps 200 --warmup 5 \
      > $out/${cfg}_cpw$cpw.json 2> $out/${cfg}_cpw$cpw.err || exit 1
  done
done
