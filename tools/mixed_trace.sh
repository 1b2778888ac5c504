# Kernel and memory-copy trace of the config-5 bench line (the tree's library): per-step GPU work.
set -e
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
GCK_AQL_TIMED=0 timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/tr" -o tr --output-format csv -- \
  python3 bench.py --config mixed --steps 40 --warmup 5 --no-cpu --no-oracle > "$OUT/tr.json" 2> "$OUT/tr.err" \
  || { tail -20 "$OUT/tr.err"; exit 1; }
python3 tools/step_trace.py "$OUT/tr" > "$OUT/step_trace.txt"
head -60 "$OUT/step_trace.txt"
find "$OUT/tr" -name "*trace.csv" -size +20M -delete
