# Per-bundle phase timing (make TIMING=1 build on the box) of one bench configuration.
# Usage on the GPU box: bash tools/timing.sh <out dir> [bench flags]
set -e
OUT=$1; shift
mkdir -p "$OUT"
touch gochugaru_amd/csrc/bundle.inc && make -C gochugaru_amd/csrc TIMING=1 > /dev/null
rm -f "$OUT/t.bin"
GCK_DEBUG_TIMING=$OUT/t timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --no-oracle "$@" > "$OUT/t.json" 2> "$OUT/t.err"
python tests/analyze_timing.py "$OUT/t.bin" > "$OUT/t.txt"
cat "$OUT/t.txt"
touch gochugaru_amd/csrc/bundle.inc && make -C gochugaru_amd/csrc > /dev/null
rm -f "$OUT/t.bin"
