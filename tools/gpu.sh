# GPU-box jobs in one parameterised tool (run under gpurun from the repo root; libraries are built
# beforehand in the container). Every GPU step has its own time limit; a failing step ends the job.
#
#   bash tools/gpu.sh tests <tag> [pytest args]          pytest -m gpu (or the given files)
#   bash tools/gpu.sh bench <tag> [bench args]           one bench.py line -> gpurun_out/<tag>/bench.json
#   bash tools/gpu.sh sweep <tag> "<flags>" ...          one bench line per flag set (no oracle / CPU)
#   bash tools/gpu.sh profile <tag> [bench args]         rocprofv3 kernel trace + stats (8 in flight and
#                                                        1 in flight), then FETCH_SIZE and WRITE_SIZE
#                                                        passes (separate runs), the gather-probe
#                                                        calibration, and traffic.json
#   bash tools/gpu.sh phases <tag> [bench args]          bench with GCK_DEBUG_PHASES=1 (snapshot / Watch
#                                                        phase times on stderr)
#   bash tools/gpu.sh pmcprobe <tag> [bench args]        one FETCH_SIZE pass over the AQL path (GCK_DEBUG_AQL)
#   bash tools/gpu.sh final <tag>                        the round-end set: pytest -m gpu, smoke, the
#                                                        driver-sized headline (twice), 2000 steps, config 5
#                                                        (20 and 500 steps), and the headline's kernel trace
#   bash tools/gpu.sh mixed <tag> [bench args]           config 5 with the Watch phases (GCK_DEBUG_PHASES)
#   bash tools/gpu.sh probes <tag>                       host-link placement (tools/pcie_probe), the
#                                                        host-batch timeline (tools/host_probe.py), the
#                                                        Watch grouping (tools/group_bench), the AQL span
#                                                        attribution (tools/aql_span.sh)
# (GCK_DEBUG_* switches act only in the debug build, make -C gochugaru_amd/csrc DEBUG=1 ->
# gochugaru_amd/libgck_debug.so: the phases / mixed / pmcprobe jobs load it through GCK_LIBRARY)
set -e
CMD=$1
TAG=$2
shift 2 || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
case "$CMD" in
  tests)
    ARGS=${*:-tests -m gpu}
    timeout -k 10 900 python -u -m pytest $ARGS -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
      || { tail -40 "$OUT/pytest.log"; exit 1; }
    tail -3 "$OUT/pytest.log"
    ;;
  bench)
    timeout -k 10 600 python3 bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
    tail -c 600 "$OUT/bench.json"
    ;;
  phases)
    GCK_LIBRARY=$PWD/gochugaru_amd/libgck_debug.so GCK_DEBUG_PHASES=1 timeout -k 10 600 python3 bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" \
      || { tail -20 "$OUT/bench.err"; exit 1; }
    grep "\[gck" "$OUT/bench.err" | tail -20
    ;;
  sweep)
    i=0
    for cfg in "$@"; do
      i=$((i+1))
      timeout -k 10 300 python3 bench.py --no-oracle --no-cpu $cfg > "$OUT/s$i.json" 2> "$OUT/s$i.err"
      echo "$cfg :: $(python3 -c "import json; d=json.load(open('$OUT/s$i.json')); print(d['value'], d.get('host_buffers', {}).get('value'))")"
    done
    ;;
  profile)
    GP=tools/gather_probe/gather_probe
    if [ -x $GP ]; then
      timeout -k 10 120 $GP > "$OUT/gather_plain.jsonl"
      timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/gfetch" -o gfetch --output-format csv -- $GP > "$OUT/gather_fetch.jsonl" 2> "$OUT/gather_fetch.err"
      timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/gwrite" -o gwrite --output-format csv -- $GP > "$OUT/gather_write.jsonl" 2> "$OUT/gather_write.err"
      echo "calibration done"
    fi
    # (under the tracer the queues' dispatch timestamps are not the packets' own: the bench's solo
    # phase is launched through HIP and timed by its events, GCK_AQL_TIMED=0; the timed region and
    # the trace are the AQL-dispatched joins)
    GCK_AQL_TIMED=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- python3 bench.py --no-cpu --host-steps 0 "$@" > "$OUT/kt.json" 2> "$OUT/kt.err"
    GCK_AQL_TIMED=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/kt1" -o kt1 --output-format csv -- python3 bench.py --no-cpu --host-steps 0 --inflight 1 "$@" > "$OUT/kt1.json" 2> "$OUT/kt1.err"
    echo "kernel trace done"
    # counter passes over the path the bench times: the joins dispatched into the engine's own HSA
    # queues (aql.inc), one batch at a time; GCK_DEBUG_AQL reports a dispatch that would stall
    SHORT="python3 bench.py --steps 20 --warmup 3 --no-oracle --no-cpu --host-steps 0 --inflight 1 $*"
    GCK_DEBUG_AQL=1 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- $SHORT > "$OUT/fetch.json" 2> "$OUT/fetch.err"
    echo "fetch pass done"
    GCK_DEBUG_AQL=1 timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- $SHORT > "$OUT/write.json" 2> "$OUT/write.err"
    echo "pmc done"
    python3 tools/traffic_summary.py "$OUT" > "$OUT/traffic.json" || true
    cat "$OUT/traffic.json" || true
    # keep the summaries; drop per-dispatch traces (gpurun_out copies back at most 64 MiB)
    find "$OUT" -name "*kernel_trace.csv" -delete
    find "$OUT" -name "*counter_collection.csv" -delete
    find "$OUT" -name "*agent_info.csv" -delete
    ;;
  pmcprobe)
    # a counter pass over the AQL path itself (the engine's own HSA queues), with the dispatch / wait
    # diagnostics of GCK_DEBUG_AQL on stderr; killed after 120 s if it stalls (run it last)
    SHORT="python3 bench.py --steps 20 --warmup 3 --no-oracle --no-cpu --host-steps 0 --inflight 1 $*"
    GCK_LIBRARY=$PWD/gochugaru_amd/libgck_debug.so GCK_DEBUG_AQL=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/aqlfetch" -o aqlfetch --output-format csv -- $SHORT > "$OUT/aqlfetch.json" 2> "$OUT/aqlfetch.err"
    rc=$?
    echo "pmc pass on the AQL path: status $rc"
    grep "gck aql" "$OUT/aqlfetch.err" | head -30 || true
    tail -5 "$OUT/aqlfetch.err"
    find "$OUT" -name "*kernel_trace.csv" -delete
    find "$OUT" -name "*agent_info.csv" -delete
    exit $rc
    ;;
  final)
    set +e
    timeout -k 10 700 python -u -m pytest -m gpu -q -rf --timeout 300 --timeout-method thread tests/ > "$OUT/pytest.log" 2>&1
    rc=$?
    echo "pytest rc=$rc" >> "$OUT/pytest.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
    set -e
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
    for r in 1 2; do
      timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver$r.json" 2> "$OUT/bench_driver$r.err"
    done
    timeout -k 10 300 python3 bench.py --no-cpu > "$OUT/bench_2000.json" 2> "$OUT/bench_2000.err"
    timeout -k 10 300 python3 bench.py --config mixed --steps 20 --warmup 5 > "$OUT/mixed20.json" 2> "$OUT/mixed20.err"
    timeout -k 10 400 python3 bench.py --config mixed --steps 500 --no-cpu > "$OUT/mixed500.json" 2> "$OUT/mixed500.err"
    timeout -k 10 300 python3 bench.py --config gdocs --steps 20 --warmup 5 > "$OUT/gdocs20.json" 2> "$OUT/gdocs20.err"
    timeout -k 10 400 python3 bench.py --config github --steps 20 --warmup 5 > "$OUT/github20.json" 2> "$OUT/github20.err"
    GCK_AQL_TIMED=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- \
      python3 bench.py --steps 20 --warmup 5 --no-cpu > "$OUT/kt.json" 2> "$OUT/kt.err"
    find "$OUT" -name "*kernel_trace.csv" -delete
    find "$OUT" -name "*agent_info.csv" -delete
    tail -2 "$OUT/pytest.log"
    ;;
  mixed)
    GCK_LIBRARY=$PWD/gochugaru_amd/libgck_debug.so GCK_DEBUG_PHASES=1 timeout -k 10 400 python3 bench.py --config mixed "$@" > "$OUT/mixed.json" 2> "$OUT/mixed.err" \
      || { tail -20 "$OUT/mixed.err"; exit 1; }
    grep "gck watch\]\|gck apply\]\|gck relink\|gck group\|apply_publish" "$OUT/mixed.err" | tail -5
    ;;
  probes)
    timeout -k 10 120 tools/pcie_probe/pcie_probe > "$OUT/pcie_probe.jsonl" 2> "$OUT/pcie_probe.err"
    timeout -k 10 200 python3 tools/host_probe.py > "$OUT/host_probe.json" 2> "$OUT/host_probe.err"
    timeout -k 10 120 tools/group_bench/group_bench 9844 400 > "$OUT/group_bench.json"
    bash tools/aql_span.sh "$OUT/aql_span"
    ;;
  *)
    echo "usage: tools/gpu.sh tests|bench|sweep|profile|phases|pmcprobe|final|mixed|probes <tag> [args]" >&2
    exit 2
    ;;
esac
