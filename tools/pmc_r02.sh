# Round-2 profile set (run on the GPU box, binaries built beforehand in this container):
#   bash tools/pmc_r02.sh <out dir under gpurun_out> [bench args]
# 1. FETCH_SIZE / WRITE_SIZE calibration on known byte counts (tools/gather_probe)
# 2. rocprofv3 kernel trace + stats of the default bench command
# 3. FETCH_SIZE and WRITE_SIZE passes (separate runs) over a short bench command
set -e
OUT=${1:-gpurun_out/pmc}
shift || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
GP=tools/gather_probe/gather_probe
timeout -k 10 120 $GP > "$OUT/gather_plain.jsonl"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/gfetch" -o gfetch --output-format csv -- $GP > "$OUT/gather_fetch.jsonl" 2> "$OUT/gather_fetch.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/gwrite" -o gwrite --output-format csv -- $GP > "$OUT/gather_write.jsonl" 2> "$OUT/gather_write.err"
echo "calibration done"
# (the CPU baseline and the host-buffer runs are left out under the tracer: they add minutes and
# nothing to the kernel statistics)
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- python3 bench.py --no-cpu --host-steps 0 "$@" > "$OUT/kt.json" 2> "$OUT/kt.err"
find "$OUT/kt" -name "*kernel_trace.csv" -delete
# one batch at a time: every launch alone on the GPU, as the bench's roofline times it
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/kt1" -o kt1 --output-format csv -- python3 bench.py --no-cpu --host-steps 0 --inflight 1 "$@" > "$OUT/kt1.json" 2> "$OUT/kt1.err"
find "$OUT/kt1" -name "*kernel_trace.csv" -delete
echo "kernel trace done"
# one batch at a time under the counters (each kernel is counted alone anyway)
SHORT="python3 bench.py --steps 20 --warmup 3 --no-oracle --no-cpu --host-steps 0 --inflight 1 $*"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- $SHORT > "$OUT/fetch.json" 2> "$OUT/fetch.err"
echo "fetch pass done"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- $SHORT > "$OUT/write.json" 2> "$OUT/write.err"
echo "pmc done"
python3 tools/traffic_summary.py "$OUT" > "$OUT/traffic.json"
cat "$OUT/traffic.json"
# keep the summaries (kernel stats, counter totals via traffic.json); drop the per-dispatch traces so
# that gpurun_out stays under the 64 MiB copy-back limit
find "$OUT" -name "*kernel_trace.csv" -delete
find "$OUT" -name "*counter_collection.csv" -delete
find "$OUT" -name "*agent_info.csv" -delete
