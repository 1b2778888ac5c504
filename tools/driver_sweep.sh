# bench.py variants in fresh processes (as the driver runs it): submit loop, batches in flight,
# hardware queues, engine-owned streams (config 4, device batches).
# Usage on the GPU box: bash tools/driver_sweep.sh <out dir> <steps> "<driver inflight queues engine_streams>"...
set -e
OUT=${1:-gpurun_out/driver_sweep}
STEPS=${2:-2000}
shift 2 || true
mkdir -p "$OUT"
SPECS=("$@")
[ ${#SPECS[@]} -gt 0 ] || SPECS=("native 3 0 0" "python 3 0 0" "native 5 0 0" "native 3 0 1" "native 5 0 1")
for rep in 1 2; do
  for spec in "${SPECS[@]}"; do
    set -- $spec
    f="$OUT/$1_$2_q$3_es$4_r$rep"
    timeout -k 10 180 python3 bench.py --no-cpu --host-steps 0 --steps "$STEPS" --warmup 100 --driver "$1" \
      --inflight "$2" --hw-queues "$3" --engine-streams "$4" > "$f.json" 2> "$f.err"
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']/1e9,3), d['ms_per_step'], d['roofline']['mean_launch_ms'])" "$f.json"
  done
done
