# A/B of one GPU test against the previous commit's library (_ab/, a worktree built in the container)
# and the current one: bash tools/ab_rev.sh <tag> <pytest node id>
set -e
TAG=$1
T=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
set +e
GCK_LIBRARY=$PWD/_ab/gochugaru_amd/libgck.so timeout -k 10 120 python -u -m pytest "$T" -x -v --timeout 100 \
  --timeout-method thread > "$OUT/old.log" 2>&1
echo "old lib: rc=$?"
tail -3 "$OUT/old.log"
timeout -k 10 120 python -u -m pytest "$T" -x -v --timeout 100 --timeout-method thread > "$OUT/new.log" 2>&1
echo "new lib: rc=$?"
tail -3 "$OUT/new.log"
