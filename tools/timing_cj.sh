# Closure-join per-wave timing with the instrumented library built beforehand here
# (make -C gochugaru_amd/csrc TIMING=1). Usage on the GPU box: bash tools/timing_cj.sh <out> [bench flags]
set -e
OUT=$1; shift
mkdir -p "$OUT"
rm -f "$OUT/t.bin" "$OUT/t_cj.bin"
GCK_LIBRARY=$PWD/gochugaru_amd/libgck_timing.so GCK_DEBUG_TIMING=$OUT/t timeout -k 10 300 \
  python bench.py --steps 10 --warmup 2 --no-cpu --no-oracle --host-steps 0 "$@" > "$OUT/t.json" 2> "$OUT/t.err"
python tools/analyze_cj.py "$OUT/t_cj.bin" > "$OUT/cj.txt"
cat "$OUT/cj.txt"
rm -f "$OUT/t.bin" "$OUT/t_cj.bin"
