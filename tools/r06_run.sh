# Round-6 GPU job: tests, then bench lines (each step under its own time limit; a failing step ends
# the job). Usage on the GPU box (from the repo root): bash tools/r06_run.sh <tag> <step>...
#   steps: tests | resident | bench64 | bench8k | bench16k | res64 | res8k | res16k | mixed | final
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
        tests/test_gpu_concurrency.py tests/test_gpu_partition.py tests/test_gpu_watch_fuzz.py -x -q --timeout 200 \
        --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
      tail -2 "$OUT/pytest.log" ;;
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
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
