# HBM traffic of the bundle kernels (rocprofv3 PMC, one counter group per pass, MI355X_MICROARCH.md
# §HBM: FETCH_SIZE doubled for gfx950) plus a kernel-trace summary of the same bench command.
# Usage on the GPU box: bash tools/pmc_traffic.sh <out dir under gpurun_out>
set -e
OUT=${1:-gpurun_out/traffic}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
CMD="python3 bench.py --steps 5 --warmup 2 --no-oracle"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- $CMD > "$OUT/kt.json" 2> "$OUT/kt.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- $CMD > "$OUT/fetch.json" 2> "$OUT/fetch.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- $CMD > "$OUT/write.json" 2> "$OUT/write.err"
python3 tools/traffic_summary.py "$OUT" > "$OUT/traffic.json"
