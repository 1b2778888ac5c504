# Address translation, L2 latency and hit-rate counters of the check kernels, one counter group
# per rocprofv3 pass. Usage on the GPU box: bash tools/pmc_lat.sh <out dir under gpurun_out> [bench args]
set -e
OUT=${1:-gpurun_out/lat}
shift || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
i=0
for ctrs in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum" \
            "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" "TCC_HIT_sum TCC_MISS_sum" \
            "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs -d "$OUT/p$i" -o p$i --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-oracle --host-steps 0 "$@" > "$OUT/p$i.json" 2> "$OUT/p$i.err"
done
python3 tools/pmc_kernel_summary.py "$OUT" > "$OUT/summary.json"
cat "$OUT/summary.json"
find "$OUT" -name "*counter_collection.csv" -delete
