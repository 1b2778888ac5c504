#!/bin/bash
# r04: the GPU suite and smoke; configs 4 / 2 / 3 with the items requested beside the table; a
# kernel trace of config 5 (the label join's stage A against the bundles).
set -o pipefail
out=gpurun_out/j10
mkdir -p $out
timeout -k 10 700 python -u -m pytest -m gpu -q -rf --timeout 300 --timeout-method thread tests/ > $out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $out/bench_driver.json 2> $out/bench_driver.err || exit 3
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 100 --no-cpu > $out/bench_2000.json 2> $out/bench_2000.err || exit 4
for cfg in gdocs github; do
  timeout -k 10 240 python -u bench.py --config $cfg --steps 200 --warmup 5 > $out/$cfg.json 2> $out/$cfg.err || exit 5
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/kt_mixed -o kt --output-format csv -- \
  python3 bench.py --config mixed --steps 20 --warmup 5 --no-cpu > $out/kt_mixed.json 2> $out/kt_mixed.err || exit 6
find $out -name "*kernel_trace.csv" -delete
find $out -name "*agent_info.csv" -delete
