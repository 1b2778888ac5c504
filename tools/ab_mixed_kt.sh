# Kernel traces of the config-5 bench line with the previous commit's library (ab_head) and the tree's.
set -e
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for v in A B; do
  if [ $v = A ]; then L=$PWD/gochugaru_amd/ab_head/libgck.so; else L=$PWD/gochugaru_amd/libgck.so; fi
  GCK_LIBRARY=$L GCK_AQL_TIMED=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/kt$v" -o kt --output-format csv -- \
    python3 bench.py --config mixed --steps 20 --warmup 5 --no-cpu --no-oracle > "$OUT/kt$v.json" 2> "$OUT/kt$v.err" \
    || { tail -20 "$OUT/kt$v.err"; exit 1; }
  find "$OUT/kt$v" -name "*kernel_trace.csv" -delete
  python3 - "$OUT/kt$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    if r["Name"].startswith("void at::") or "elementwise" in r["Name"]: continue
    print(r["Name"][:50], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
PY
done
