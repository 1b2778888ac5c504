#!/bin/bash
# r04: the label join stages its slot lines in two phases (LDS 28 -> 20 KB per block at 32 words:
# 6-7 blocks per CU instead of 5); label / parity / config tests; configs 2, 3 twice; config 5.
set -o pipefail
out=gpurun_out/j41
mkdir -p $out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_labels.py \
  tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_partition.py tests/test_gpu_slots.py > $out/pytest.log 2>&1 || exit 1
for r in 1 2; do
  for cfg in gdocs github; do
    timeout -k 10 240 python -u bench.py --config $cfg --steps 200 --warmup 5 > $out/${cfg}_$r.json 2> $out/${cfg}_$r.err || exit 2
  done
done
timeout -k 10 300 python -u bench.py --config mixed --steps 20 --warmup 5 --no-cpu > $out/mixed.json 2> $out/mixed.err || exit 3
