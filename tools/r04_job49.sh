#!/bin/bash
# r04 (late): the GPU suite, smoke, the headline bench (driver-sized and 2000 steps) and its kernel trace.
set -o pipefail
out=gpurun_out/j49
mkdir -p $out
timeout -k 10 700 python -u -m pytest -m gpu -q -rf --timeout 300 --timeout-method thread tests/ > $out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $out/bench_driver.json 2> $out/bench_driver.err || exit 3
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > $out/bench_driver2.json 2> $out/bench_driver2.err || exit 3
timeout -k 10 300 python -u bench.py --config mixed --steps 20 --warmup 5 > $out/mixed.json 2> $out/mixed.err || exit 3
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 100 --no-cpu > $out/bench_2000.json 2> $out/bench_2000.err || exit 4
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
GCK_AQL_TIMED=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/kt -o kt --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu --host-steps 0 > $out/kt.json 2> $out/kt.err || exit 5
find $out -name "*kernel_trace.csv" -delete
find $out -name "*agent_info.csv" -delete
find $out -type f -size +4M -delete
