#!/bin/bash
# r04: wave bundles sized to the list (a short chained list over every slot); kernarg lines
# written only when changed. Parity + labels + concurrency; configs 5, 2, 3, 4.
set -o pipefail
out=gpurun_out/j18
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_labels.py tests/test_gpu_concurrency.py tests/test_aql_codeobject.py > $out/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config mixed --steps 20 --warmup 5 > $out/mixed.json 2> $out/mixed.err || exit 3
for cfg in gdocs github; do
  GCK_DEBUG_PHASES=1 timeout -k 10 240 python -u bench.py --config $cfg --steps 200 --warmup 5 > $out/$cfg.json 2> $out/$cfg.err || exit 2
done
timeout -k 10 240 python -u bench.py > $out/default.json 2> $out/default.err || exit 4
timeout -k 10 240 python -u bench.py --steps 2000 --warmup 20 > $out/long.json 2> $out/long.err || exit 5
