#!/bin/bash
# r04: label tables under config 5's churn (wildcard grants defer their resource), level bounds
# from the sorted levels; tests first, then config 5 with phases, the driver-sized config 5 run,
# the nesting Watch at 1e9.
set -o pipefail
out=gpurun_out/j6
mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_labels.py \
  tests/test_gpu_mixed.py tests/test_gpu_delta.py tests/test_gpu_scale.py \
  "tests/test_gpu_fullsize.py::test_config5_full_with_three_watch_batches" > $out/pytest.log 2>&1 || exit 1
GCK_DEBUG_PHASES=1 timeout -k 10 200 python -u bench.py --config mixed --steps 4 --warmup 2 --no-cpu \
  > $out/mixed_phases.json 2> $out/mixed_phases.err || exit 2
timeout -k 10 200 python -u bench.py --config mixed --steps 20 --warmup 5 > $out/bench_mixed.json 2> $out/bench_mixed.err || exit 3
GCK_DEBUG_PHASES=1 timeout -k 10 240 python -u tools/watch_bench.py --tuples 1e9 --batches 2 --mix nesting --verify \
  > $out/wb_nesting.log 2>&1 || exit 4
