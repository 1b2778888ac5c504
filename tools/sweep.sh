# Parameter sweep of the bench (no oracle, no CPU baseline): one JSON line per config.
# Usage on the GPU box: bash tools/sweep.sh <out dir> "<flags 1>" "<flags 2>" ...
set -e
OUT=$1; shift
mkdir -p "$OUT"
i=0
for cfg in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-oracle $cfg > "$OUT/s$i.json" 2> "$OUT/s$i.err"
  echo "$cfg :: $(python -c "import json,sys; d=json.load(open('$OUT/s$i.json')); print(d['value'], d['engine'])")"
done
