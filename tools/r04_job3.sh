#!/bin/bash
# r04: the GPU suite, then the 1e9 Watch benches (membership-only, nesting) and config 5.
# A test failure (pytest status 1) does not stop the measurements; a crash, abort or time limit does.
set -o pipefail
out=gpurun_out/j3
mkdir -p $out
timeout -k 10 700 python -u -m pytest -m gpu -q -rf --timeout 300 --timeout-method thread tests/ > $out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
GCK_DEBUG_PHASES=1 timeout -k 10 240 python -u tools/watch_bench.py --tuples 1e9 --batches 3 --mix members --verify \
  > $out/wb_members.log 2>&1 || exit 2
GCK_DEBUG_PHASES=1 timeout -k 10 240 python -u tools/watch_bench.py --tuples 1e9 --batches 2 --mix nesting --verify \
  > $out/wb_nesting.log 2>&1 || exit 3
timeout -k 10 200 python -u bench.py --config mixed --steps 20 --warmup 5 > $out/bench_mixed.json 2> $out/bench_mixed.err || exit 4
