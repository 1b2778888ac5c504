# Configs 2 / 3 through the rotated-batch loop: batches in flight x engine streams (fresh processes).
# Usage on the GPU box: bash tools/configs_sweep.sh <out dir under gpurun_out>
set -e
OUT=${1:-gpurun_out/configs_sweep}
mkdir -p "$OUT"
for c in gdocs github; do
  for spec in "3 0" "3 1" "8 1" "16 1"; do
    set -- $spec
    f="$OUT/${c}_$1_es$2"
    timeout -k 10 300 python3 bench.py --config $c --no-cpu --host-steps 0 --steps 400 --warmup 40 --inflight $1 \
      --engine-streams $2 > "$f.json" 2> "$f.err"
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']/1e6,1), 'M', d['ms_per_step'], d.get('oracle_agreement'))" "$f.json"
  done
done
