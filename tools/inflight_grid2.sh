# Distinct rotated batches, Python and compiled loops alternating in one process (config 4 graph).
# Usage on the GPU box: bash tools/inflight_grid2.sh <out dir under gpurun_out>
set -e
OUT=${1:-gpurun_out/inflight_grid2}
mkdir -p "$OUT"
for ws in 8; do
  timeout -k 10 240 python3 tools/inflight_probe.py --both --rot 2100 --reps 2 --batches 2000 --depths 3,4,5,8 \
    --workspaces $ws > "$OUT/ws$ws.txt" 2> "$OUT/ws$ws.err"
  echo "ws=$ws"; cat "$OUT/ws$ws.txt"
done
