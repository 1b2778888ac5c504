# engine-stream wait cost + partitioned level loop with fewer host synchronisations
set -e
OUT=${1:-gpurun_out/r02c}
mkdir -p "$OUT"
bash tools/driver_sweep.sh "$OUT/sweep" 2000 "native 16 0 1" "native 8 0 1"
timeout -k 10 400 python3 bench.py --partitioned --no-cpu --host-steps 0 --steps 20 --warmup 3 > "$OUT/part.json" 2> "$OUT/part.err"
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('partitioned', d['value'], d['ms_per_step'], d['oracle_agreement'])" "$OUT/part.json"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_partition.py tests/test_gpu_concurrency.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
tail -2 "$OUT/pytest.log"
