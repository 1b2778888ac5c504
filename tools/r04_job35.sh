#!/bin/bash
# r04: a context batch whose dense caveat table the workspace already holds uploads nothing.
set -o pipefail
out=gpurun_out/j35
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_labels.py \
  tests/test_gpu_caveat_scale.py tests/test_gpu_cel.py tests/test_gpu_mixed.py tests/test_gpu_parity.py -k "cav or Cav or context or mixed or caveat" > $out/pytest.log 2>&1 || exit 1
for r in 1 2; do
timeout -k 10 300 python -u bench.py --config mixed --steps 20 --warmup 5 --no-cpu > $out/mixed_$r.json 2> $out/mixed_$r.err || exit 2
done
