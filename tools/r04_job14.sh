#!/bin/bash
# r04: packed slots chosen per snapshot — label tests, configs 2, 3, 5.
set -o pipefail
out=gpurun_out/j14
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_labels.py \
  tests/test_gpu_configs.py tests/test_gpu_partition.py > $out/pytest.log 2>&1 || exit 1
for cfg in gdocs github; do
  GCK_DEBUG_PHASES=1 timeout -k 10 240 python -u bench.py --config $cfg --steps 200 --warmup 5 > $out/$cfg.json 2> $out/$cfg.err || exit 2
done
timeout -k 10 300 python -u bench.py --config mixed --steps 20 --warmup 5 > $out/mixed.json 2> $out/mixed.err || exit 3
