#!/bin/bash
# r04: resource slots of 24-bit fields — the label-join tests (parity families, partitions,
# caveat plane, full-size configs 2/3/5), then configs 2, 3 and 5 with the slot formats logged.
set -o pipefail
out=gpurun_out/j13
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_labels.py \
  tests/test_gpu_parity.py tests/test_gpu_partition.py tests/test_gpu_mixed.py tests/test_gpu_configs.py \
  "tests/test_gpu_fullsize.py::test_config2_config3_full_batch" \
  "tests/test_gpu_fullsize.py::test_config5_full_with_three_watch_batches" > $out/pytest.log 2>&1 || exit 1
for cfg in gdocs github; do
  GCK_DEBUG_PHASES=1 timeout -k 10 240 python -u bench.py --config $cfg --steps 200 --warmup 5 > $out/$cfg.json 2> $out/$cfg.err || exit 2
done
timeout -k 10 300 python -u bench.py --config mixed --steps 20 --warmup 5 > $out/mixed.json 2> $out/mixed.err || exit 3
