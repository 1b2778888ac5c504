#!/bin/bash
# r04: config 5 with and without the label join (its stage A, the Watch share), slot formats.
set -o pipefail
out=gpurun_out/j8
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_labels.py \
  tests/test_gpu_mixed.py tests/test_aql_codeobject.py > $out/pytest.log 2>&1 || exit 1
GCK_DEBUG_PHASES=1 timeout -k 10 200 python -u bench.py --config mixed --steps 20 --warmup 5 \
  > $out/mixed.json 2> $out/mixed.err || exit 2
timeout -k 10 200 python -u bench.py --config mixed --steps 20 --warmup 5 --no-labels --no-cpu \
  > $out/mixed_nolabels.json 2> $out/mixed_nolabels.err || exit 3
GCK_DEBUG_PHASES=1 timeout -k 10 200 python -u bench.py --config gdocs --steps 20 --warmup 5 --no-cpu \
  > $out/gdocs.json 2> $out/gdocs.err || exit 4
