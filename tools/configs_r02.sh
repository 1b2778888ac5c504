# BASELINE configs 2, 3, 5 (+ the config-5 caveat-scale variant) on one GPU, one bench line each.
# Usage on the GPU box: bash tools/configs_r02.sh <out dir under gpurun_out>
set -e
OUT=${1:-gpurun_out/configs}
mkdir -p "$OUT"
for c in gdocs github mixed quota; do
  timeout -k 10 400 python3 bench.py --config "$c" > "$OUT/$c.json" 2> "$OUT/$c.err"
  echo "$c done"
done
