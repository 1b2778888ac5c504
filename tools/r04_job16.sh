#!/bin/bash
# r04: kernarg lines written only when they change; the launch-path knob probe without deferrals;
# configs 2, 3 (packed slots, pipelined user scan); the headline at driver size and long.
set -o pipefail
out=gpurun_out/j16
mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_labels.py \
  tests/test_gpu_concurrency.py tests/test_aql_codeobject.py > $out/pytest.log 2>&1 || exit 1
for cfg in gdocs github; do
  GCK_DEBUG_PHASES=1 timeout -k 10 240 python -u bench.py --config $cfg --steps 200 --warmup 5 > $out/$cfg.json 2> $out/$cfg.err || exit 2
done
timeout -k 10 240 python -u bench.py > $out/default.json 2> $out/default.err || exit 3
timeout -k 10 240 python -u bench.py --steps 2000 --warmup 20 > $out/long.json 2> $out/long.err || exit 4
