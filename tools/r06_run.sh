# Round-6 GPU job: tests, then bench lines (each step under its own time limit; a failing step ends
# the job). Usage on the GPU box (from the repo root): bash tools/r06_run.sh <tag> <step>...
#   steps: tests | chain | chunk | resident | bench64 | bench8k | bench16k | res64 | res8k | res16k | mixed |
#          mixed2k | phases | pmc_nested | pmc_gdocs | pmc_github | pmc_mixed
set -e
TAG=$1
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
b() {  # one bench line: b <name> <seconds> <args...>
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" python3 bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail -20 "$OUT/$name.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], (d.get('baseline_pipelined') or {}).get('value'), (d.get('baseline_pipelined_uniform') or {}).get('value'), (d.get('roofline') or {}).get('frac'), d['engine'].get('resident_batches'), d.get('oracle_agreement'))"
}
for step in "$@"; do
  case "$step" in
    tests)
      timeout -k 10 1000 python -u -m pytest tests/test_gpu_uniform.py tests/test_gpu_parity.py tests/test_gpu_hostpath.py \
        tests/test_gpu_concurrency.py tests/test_gpu_partition.py tests/test_gpu_watch_fuzz.py -x -v --timeout 120 \
        --timeout-method thread \
        > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
      tail -2 "$OUT/pytest.log" ;;
    chain)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_mixed.py tests/test_gpu_labels.py -x -v --timeout 300 \
        --timeout-method thread > "$OUT/pytest_chain.log" 2>&1 || { tail -40 "$OUT/pytest_chain.log"; exit 1; }
      tail -2 "$OUT/pytest_chain.log" ;;
    chunkp)
      timeout -k 10 150 python -u -m pytest tests/test_gpu_uniform.py::test_uniform_chunks_above_max_batch -x -v -s \
        --timeout 100 --timeout-method thread > "$OUT/pytest_chunkp.log" 2>&1 || { tail -60 "$OUT/pytest_chunkp.log"; exit 1; }
      tail -2 "$OUT/pytest_chunkp.log" ;;
    resdbg)
      GCK_LIBRARY=$PWD/gochugaru_amd/libgck_debug.so GCK_DEBUG_RES=1 timeout -k 10 300 python -u -m pytest \
        tests/test_gpu_resident.py -x -v -s --timeout 120 --timeout-method thread > "$OUT/pytest_resdbg.log" 2>&1
      echo "resdbg rc=$?"; grep "gck res" "$OUT/pytest_resdbg.log" | sort | uniq -c | sort -rn | head -8; tail -2 "$OUT/pytest_resdbg.log" ;;
    watch)
      timeout -k 10 900 python -u -m pytest tests/test_gpu_delta.py tests/test_gpu_watch_fuzz.py tests/test_gpu_watch_nested.py \
        tests/test_gpu_watch_concurrent.py tests/test_gpu_resident.py -x -v --timeout 300 --timeout-method thread \
        > "$OUT/pytest_watch.log" 2>&1 || { tail -40 "$OUT/pytest_watch.log"; exit 1; }
      tail -2 "$OUT/pytest_watch.log" ;;
    fs4)
      timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -k "config4_1e9_full_batch" -x -v -s --timeout 800 \
        --timeout-method thread > "$OUT/pytest_fs4.log" 2>&1 || { tail -40 "$OUT/pytest_fs4.log"; exit 1; }
      grep "footprint" "$OUT/pytest_fs4.log"; tail -2 "$OUT/pytest_fs4.log" ;;
    ljtime) timeout -k 10 400 bash tools/timing_lj.sh "$OUT/ljt" --config mixed ;;
    qsweep)  # 8,192-check requests: queues x requests in flight (the debug library's queue-count switch)
      for qi in "4 16" "8 16" "8 32"; do
        set -- $qi
        GCK_LIBRARY=$PWD/gochugaru_amd/libgck_debug.so GCK_DEBUG_AQL_QUEUES=$1 timeout -k 10 300 python3 bench.py \
          --batch 8192 --steps 1000 --inflight $2 --no-cpu --no-oracle --host-steps 0 > "$OUT/q$1_if$2.json" 2> "$OUT/q$1_if$2.err" \
          || { tail -5 "$OUT/q$1_if$2.err"; exit 1; }
        echo "queues=$1 inflight=$2 $(python3 -c "import json; print(json.load(open('$OUT/q$1_if$2.json'))['value'])")"
      done ;;
    chunk)
      GCK_LIBRARY=$PWD/gochugaru_amd/libgck_debug.so GCK_DEBUG_AQL=1 timeout -k 10 150 python -u -m pytest \
        tests/test_gpu_uniform.py::test_uniform_chunks_above_max_batch -x -v -s --timeout 100 --timeout-method thread \
        > "$OUT/pytest_chunk.log" 2>&1 || { tail -60 "$OUT/pytest_chunk.log"; exit 1; }
      tail -2 "$OUT/pytest_chunk.log" ;;
    resident)
      timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py -x -v --timeout 120 --timeout-method thread \
        > "$OUT/pytest_resident.log" 2>&1 || { tail -40 "$OUT/pytest_resident.log"; exit 1; }
      tail -2 "$OUT/pytest_resident.log" ;;
    bench64) b bench64 400 --steps 200 ;;
    bench8k) b bench8k 400 --batch 8192 --steps 1000 --no-cpu ;;
    bench16k) b bench16k 400 --batch 16384 --steps 1000 --no-cpu ;;
    res64) b res64 400 --steps 200 --resident 1 --no-cpu ;;
    res8k) b res8k 400 --batch 8192 --steps 1000 --no-cpu --resident 1 ;;
    res16k) b res16k 400 --batch 16384 --steps 1000 --no-cpu --resident 1 ;;
    mixed) b mixed 400 --config mixed --steps 20 --warmup 5 ;;
    mixed2k) b mixed2k 600 --config mixed --steps 2000 --no-cpu ;;
    phases) bash tools/gpu.sh mixed "${TAG}_phases" --steps 200 --no-cpu ;;
    pmc_nested) bash tools/gpu.sh profile "${TAG}_pmc_nested" ;;
    pmc_gdocs) bash tools/gpu.sh profile "${TAG}_pmc_gdocs" --config gdocs ;;
    pmc_github) bash tools/gpu.sh profile "${TAG}_pmc_github" --config github ;;
    pmc_mixed) bash tools/gpu.sh profile "${TAG}_pmc_mixed" --config mixed ;;
    part) b part 600 --partitioned --steps 100 --warmup 5 --no-cpu ;;
    partkt)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/part_kt" -o kt --output-format csv -- \
        python3 bench.py --partitioned --steps 100 --warmup 5 --no-cpu --no-oracle > "$OUT/part_kt.json" 2> "$OUT/part_kt.err" \
        || { tail -20 "$OUT/part_kt.err"; exit 1; }
      find "$OUT/part_kt" -name "*kernel_trace.csv" -delete
      find "$OUT/part_kt" -name "*agent_info.csv" -delete ;;
    endbench)  # the round-end bench lines: the driver's default twice, 2,000 steps, configs 2 / 3 / 5
      b driver1 300 --gpus 1 --steps 20 --warmup 5
      b driver2 300 --gpus 1 --steps 20 --warmup 5
      b bench2000 300 --no-cpu
      b mixed20 300 --config mixed --steps 20 --warmup 5
      b mixed500 400 --config mixed --steps 500 --no-cpu
      b gdocs20 300 --config gdocs --steps 20 --warmup 5
      b github20 400 --config github --steps 20 --warmup 5 ;;
    endkt)
      GCK_AQL_TIMED=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- \
        python3 bench.py --steps 20 --warmup 5 --no-cpu > "$OUT/kt.json" 2> "$OUT/kt.err" || { tail -20 "$OUT/kt.err"; exit 1; }
      find "$OUT" -name "*kernel_trace.csv" -delete
      find "$OUT" -name "*agent_info.csv" -delete ;;
    full)
      timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
        > "$OUT/pytest_full.log" 2>&1 || { tail -40 "$OUT/pytest_full.log"; exit 1; }
      tail -2 "$OUT/pytest_full.log" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
