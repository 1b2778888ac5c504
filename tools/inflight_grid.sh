# Batches in flight x hardware queues x driver, one engine per process (config 4 graph).
# Usage on the GPU box: bash tools/inflight_grid.sh <out dir under gpurun_out>
set -e
OUT=${1:-gpurun_out/inflight_grid}
mkdir -p "$OUT"
for q in 4 8 16; do
  for drv in native python; do
    flag=""; [ "$drv" = native ] && flag="--native"
    timeout -k 10 240 python3 tools/inflight_probe.py --queues $q $flag --reps 2 --batches 2000 --depths 1,2,3,4,5,6,8 \
      > "$OUT/q${q}_$drv.txt" 2> "$OUT/q${q}_$drv.err"
    echo "q=$q $drv"; grep "rep 1" "$OUT/q${q}_$drv.txt"
  done
done
