#!/bin/bash
# r04: config 5 with stage A timed to the end of the chained bundles, with and without labels.
set -o pipefail
out=gpurun_out/j12
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_mixed.py \
  tests/test_gpu_labels.py tests/test_gpu_concurrency.py > $out/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config mixed --steps 20 --warmup 5 > $out/mixed.json 2> $out/mixed.err || exit 2
timeout -k 10 300 python -u bench.py --config mixed --steps 20 --warmup 5 --no-labels > $out/mixed_nolabels.json 2> $out/mixed_nolabels.err || exit 3
