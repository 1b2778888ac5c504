#!/bin/bash
# r04: the device-built ancestors at scale (2e7 deep hierarchies, the 1e9 batch), then the 1e9
# Watch benches (membership-only, nesting) and config 5. Any failure stops the script.
set -o pipefail
out=gpurun_out/j5
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_scale.py \
  "tests/test_gpu_fullsize.py::test_config4_1e9_full_batch" > $out/pytest.log 2>&1 || exit 1
GCK_DEBUG_PHASES=1 timeout -k 10 240 python -u tools/watch_bench.py --tuples 1e9 --batches 3 --mix members --verify \
  > $out/wb_members.log 2>&1 || exit 2
GCK_DEBUG_PHASES=1 timeout -k 10 240 python -u tools/watch_bench.py --tuples 1e9 --batches 2 --mix nesting --verify \
  > $out/wb_nesting.log 2>&1 || exit 3
timeout -k 10 200 python -u bench.py --config mixed --steps 20 --warmup 5 > $out/bench_mixed.json 2> $out/bench_mixed.err || exit 4
