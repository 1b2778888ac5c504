#!/bin/bash
# r04: label join sanity, then config 5 with phases over a driver-sized run (why do the tables
# rebuild?), config 5 again, and the checks-per-wave A/B on configs 2 and 3.
set -o pipefail
out=gpurun_out/j7
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_labels.py \
  tests/test_gpu_mixed.py > $out/pytest.log 2>&1 || exit 1
GCK_DEBUG_PHASES=1 timeout -k 10 200 python -u bench.py --config mixed --steps 20 --warmup 5 --no-cpu \
  > $out/mixed_phases.json 2> $out/mixed_phases.err || exit 2
timeout -k 10 200 python -u bench.py --config mixed --steps 20 --warmup 5 > $out/bench_mixed.json 2> $out/bench_mixed.err || exit 3
for cfg in gdocs github; do
  for cpw in 32 16; do
    GCK_LJ_CPW=$cpw timeout -k 10 240 python -u bench.py --config $cfg --steps 200 --warmup 5 --no-cpu \
      > $out/${cfg}_cpw$cpw.json 2> $out/${cfg}_cpw$cpw.err || exit 4
  done
done
