# Per-bundle phase timing of one bench configuration, with the instrumented library built
# beforehand here (make -C gochugaru_amd/csrc TIMING=1 -> gochugaru_amd/libgck_timing.so).
# Usage on the GPU box: bash tools/timing.sh <out dir> [bench flags]
set -e
OUT=$1; shift
mkdir -p "$OUT"
rm -f "$OUT/t.bin"
GCK_LIBRARY=$PWD/gochugaru_amd/libgck_timing.so GCK_DEBUG_TIMING=$OUT/t timeout -k 10 300 \
  python bench.py --steps 3 --warmup 1 --no-cpu --no-oracle --host-steps 0 "$@" > "$OUT/t.json" 2> "$OUT/t.err"
python tools/analyze_timing.py "$OUT/t.bin" > "$OUT/t.txt"
cat "$OUT/t.txt"
rm -f "$OUT/t.bin"
