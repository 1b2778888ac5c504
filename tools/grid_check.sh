# Grid-wide path changes: partitioned config 4 at one rank, configs 2 / 3, then the parity tests.
# Usage on the GPU box: bash tools/grid_check.sh <out dir under gpurun_out>
set -e
OUT=${1:-gpurun_out/grid}
mkdir -p "$OUT"
timeout -k 10 400 python3 bench.py --partitioned --no-cpu --host-steps 0 --steps 20 --warmup 3 > "$OUT/part.json" 2> "$OUT/part.err"
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('partitioned', d['value'], d['ms_per_step'], d['oracle_agreement'])" "$OUT/part.json"
for c in gdocs github; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu --host-steps 0 --steps 400 --warmup 40 > "$OUT/$c.json" 2> "$OUT/$c.err"
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']/1e6,1), 'M', d['ms_per_step'])" "$OUT/$c.json"
done
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_partition.py tests/test_gpu_caveat_scale.py tests/test_gpu_mixed.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
tail -2 "$OUT/pytest.log"
