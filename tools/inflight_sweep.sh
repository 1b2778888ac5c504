# Sweep of batches in flight (bench.py --inflight) on config 4, device-resident and PCIe-inclusive:
#   bash tools/inflight_sweep.sh <tag> [extra bench args...]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-sweep}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for d in 1 2 3 4 6 2; do
  timeout -k 10 240 python bench.py --inflight $d --steps 200 --host-steps 200 --no-cpu --no-oracle "$@" > "$OUT/inf$d.json" 2>/dev/null
  python - "$OUT/inf$d.json" $d <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")]
d = json.loads(l[-1]); h = d.get("host_buffers") or {}
print("inflight", sys.argv[2], "device %.1fM" % (d["value"] / 1e6), "ms %.4f" % d["ms_per_step"],
      "host-pinned %.1fM" % (h.get("value", 0) / 1e6), "pageable %.1fM" % ((h.get("pageable") or {}).get("value", 0) / 1e6),
      "one %.1fM" % ((h.get("one_at_a_time") or {}).get("value", 0) / 1e6), "same", h.get("same_results"), flush=True)
PY
done
