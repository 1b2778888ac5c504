#!/bin/bash
# r04: context batches' label join through the engine's HSA queue (Ctx in the kernarg block,
# caveat flags cleared by the join); labels / caveats / concurrency / parity / mixed tests; configs 5, 5q.
set -o pipefail
out=gpurun_out/j25
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_labels.py \
  tests/test_aql_codeobject.py tests/test_gpu_concurrency.py tests/test_gpu_parity.py tests/test_gpu_mixed.py \
  tests/test_gpu_caveat_scale.py tests/test_gpu_cel.py tests/test_gpu_delta.py > $out/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config mixed --steps 20 --warmup 5 > $out/mixed.json 2> $out/mixed.err || exit 2
timeout -k 10 300 python -u bench.py --config quota --steps 20 --warmup 5 > $out/quota.json 2> $out/quota.err || exit 3
