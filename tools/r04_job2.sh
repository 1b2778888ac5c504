#!/bin/bash
# r04: Watch transposed merge + caveat plane checks (tests, then the members-only 1e9 Watch bench)
set -o pipefail
mkdir -p gpurun_out/j2
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_labels.py tests/test_gpu_delta.py tests/test_gpu_watch_nested.py tests/test_gpu_watch_concurrent.py \
  tests/test_gpu_mixed.py tests/test_gpu_parity.py tests/test_gpu_cel.py > gpurun_out/j2/pytest.log 2>&1 || exit 1
GCK_DEBUG_PHASES=1 timeout -k 10 500 python -u tools/watch_bench.py --tuples 1e9 --batches 3 --mix members --verify \
  > gpurun_out/j2/wb_members.log 2>&1 || exit 2
