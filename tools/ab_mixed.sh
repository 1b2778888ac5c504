# A/B of the config-5 bench line: the previous commit's library (gochugaru_amd/ab_head/, built in the
# container from a worktree of HEAD) against the tree's, alternated on one box.
# Usage: bash tools/ab_mixed.sh <tag> <steps> [config]
set -e
TAG=$1
STEPS=${2:-20}
CFG=${3:-mixed}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then L=$PWD/gochugaru_amd/ab_head/libgck.so; else L=$PWD/gochugaru_amd/libgck.so; fi
    GCK_LIBRARY=$L timeout -k 10 300 python3 bench.py --config "$CFG" --steps "$STEPS" --warmup 5 --no-cpu --no-oracle \
      > "$OUT/mixed_${v}$r.json" 2> "$OUT/mixed_${v}$r.err" || { tail -20 "$OUT/mixed_${v}$r.err"; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/mixed_${v}$r.json')); en=d['engine']; w=d.get('watch')
w = w or {}
print('$v$r', round(d['value']/1e6,1), 'M/s step', d['ms_per_step'], 'apply', w.get('apply_ms_per_step'), 'dev', en.get('device_ms_per_batch'), 'bund', en.get('bundles_per_batch'), 'lab', en.get('label_checks_per_batch'))"
  done
done
