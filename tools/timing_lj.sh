# Label-join per-wave timing with the instrumented library built beforehand here
# (make -C gochugaru_amd/csrc TIMING=1). Usage on the GPU box: bash tools/timing_lj.sh <out> --config gdocs|github
set -e
OUT=$1; shift
mkdir -p "$OUT"
rm -f "$OUT/t.bin" "$OUT/t_lj.bin" "$OUT/t_cj.bin"
GCK_LIBRARY=$PWD/gochugaru_amd/libgck_timing.so GCK_DEBUG_TIMING=$OUT/t timeout -k 10 300 \
  python bench.py --steps 10 --warmup 2 --no-cpu --no-oracle --host-steps 0 --inflight 1 "$@" > "$OUT/t.json" 2> "$OUT/t.err"
python tools/analyze_lj.py "$OUT/t_lj.bin" > "$OUT/lj.txt"
cat "$OUT/lj.txt"
# (the bundles the join left, when any ran: tools/analyze_timing.py)
if [ -s "$OUT/t.bin" ]; then python tools/analyze_timing.py "$OUT/t.bin" > "$OUT/bundles.txt" && cat "$OUT/bundles.txt"; fi
rm -f "$OUT/t.bin" "$OUT/t_lj.bin" "$OUT/t_cj.bin"
