#!/bin/bash
# r04: queue timestamps enabled at queue creation (solo launches timed in every process);
# configs 2, 3, 4 twice each; concurrency + AQL tests.
set -o pipefail
out=gpurun_out/j28
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_concurrency.py \
  tests/test_aql_codeobject.py > $out/pytest.log 2>&1 || exit 1
for r in 1 2; do
  for cfg in gdocs github; do
    timeout -k 10 240 python -u bench.py --config $cfg --steps 200 --warmup 5 > $out/${cfg}_$r.json 2> $out/${cfg}_$r.err || exit 2
  done
  timeout -k 10 240 python -u bench.py > $out/default_$r.json 2> $out/default_$r.err || exit 3
done
timeout -k 10 240 python -u bench.py --steps 2000 --warmup 20 > $out/long.json 2> $out/long.err || exit 4
