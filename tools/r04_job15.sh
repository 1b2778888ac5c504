#!/bin/bash
# r04: the label join's user scan pipelined; configs 2, 3 (packed slots); the launch-path knobs.
set -o pipefail
out=gpurun_out/j15
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_labels.py \
  tests/test_gpu_concurrency.py > $out/pytest.log 2>&1 || exit 1
for cfg in gdocs github; do
  GCK_DEBUG_PHASES=1 timeout -k 10 240 python -u bench.py --config $cfg --steps 200 --warmup 5 > $out/$cfg.json 2> $out/$cfg.err || exit 2
done
