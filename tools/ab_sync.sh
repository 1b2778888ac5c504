# A/B of the batch completion path on the GPU box: k_publish + host spin (default) vs
# copy + hipStreamSynchronize (GCK_SYNC_STREAM=1). Usage: bash tools/ab_sync.sh <tag>
set -e
TAG=${1:-ab}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 300 python bench.py --no-cpu > "$OUT/bench_publish.json" 2> "$OUT/bench_publish.err"
GCK_SYNC_STREAM=1 timeout -k 10 300 python bench.py --no-cpu > "$OUT/bench_stream.json" 2> "$OUT/bench_stream.err"
python - "$OUT" <<'PY'
import json, sys
for k in ("publish", "stream"):
    d = json.load(open(f"{sys.argv[1]}/bench_{k}.json"))
    print(k, d["value"], d["ms_per_step"], d["engine"]["device_ms_per_batch"], d["roofline"]["mean_launch_ms"], d.get("host_buffers"), d["oracle_agreement"])
PY
