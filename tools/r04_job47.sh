#!/bin/bash
# r04: a Watch batch waits for its merge totals only; the merge kernel runs on beside the host's
# derivation of the next snapshot. Watch / label / partition tests; config 5.
set -o pipefail
out=gpurun_out/j47
mkdir -p $out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_delta.py \
  tests/test_gpu_watch_concurrent.py tests/test_gpu_watch_nested.py tests/test_gpu_mixed.py tests/test_gpu_labels.py \
  tests/test_gpu_partition.py tests/test_gpu_scale.py > $out/pytest.log 2>&1 || exit 1
for r in 1 2; do
timeout -k 10 300 python -u bench.py --config mixed --steps 20 --warmup 5 --no-cpu > $out/mixed_$r.json 2> $out/mixed_$r.err || exit 2
done
GCK_DEBUG_PHASES=1 timeout -k 10 300 python -u bench.py --config mixed --steps 20 --warmup 5 --no-cpu > $out/mixed_ph.json 2> $out/mixed_ph.err || exit 3
