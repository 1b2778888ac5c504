# Config 2: the submit loop and streams of the default against round-2's earlier setting.
set -e
OUT=${1:-gpurun_out/gdocs_ab}
mkdir -p "$OUT"
for spec in "python 0" "native 0" "python 1" "native 1"; do
  set -- $spec
  timeout -k 10 300 python3 bench.py --config gdocs --no-cpu --host-steps 0 --driver $1 --engine-streams $2 > "$OUT/$1_$2.json" 2> "$OUT/$1_$2.err"
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'], d['engine'].get('deferred_per_batch'), d['engine'].get('closure_checks_per_batch'))" "$OUT/$1_$2.json"
done
