#!/bin/bash
# r04: the Watch batch's label marks in one launch; label / Watch tests; config 5 with phases.
set -o pipefail
out=gpurun_out/j30
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_labels.py \
  tests/test_gpu_delta.py tests/test_gpu_mixed.py tests/test_gpu_partition.py > $out/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config mixed --steps 20 --warmup 5 > $out/mixed.json 2> $out/mixed.err || exit 2
GCK_DEBUG_PHASES=1 timeout -k 10 300 python -u bench.py --config mixed --steps 20 --warmup 5 --no-cpu > $out/mixed_ph.json 2> $out/mixed_ph.err || exit 3
