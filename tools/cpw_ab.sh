# Closure join at 32 vs 64 checks per wave (GCK_CJ_CPW): slot parity tests, then the default bench.
set -e
OUT=${1:-gpurun_out/cpw}
mkdir -p "$OUT"
[ -n "$SKIP_TESTS" ] || GCK_CJ_CPW=32 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_slots.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest32.log" 2>&1
[ -n "$SKIP_TESTS" ] || tail -1 "$OUT/pytest32.log"
for rep in 1 2 3; do
  for cpw in 32 64; do
    GCK_CJ_CPW=$cpw timeout -k 10 300 python3 bench.py --no-cpu --host-steps 0 > "$OUT/b${cpw}_$rep.json" 2> "$OUT/b${cpw}_$rep.err"
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value']/1e9,3), d['ms_per_step'], d['roofline']['mean_launch_ms'], d['oracle_agreement'])" "$OUT/b${cpw}_$rep.json"
  done
done
