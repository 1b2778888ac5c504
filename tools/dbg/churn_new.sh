cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g9
T=tests/test_gpu_labels.py::test_direct_grant_churn_keeps_the_tables
GCK_LIBRARY=$PWD/gochugaru_amd/libgck_walkdbg.so timeout -k 10 200 python -u -m pytest $T -x -v -s --timeout 150 \
  --timeout-method thread > gpurun_out/g9/walk.log 2>&1
rc=$?
echo "walkdbg rc=$rc"; tail -3 gpurun_out/g9/walk.log; grep -c "^walk" gpurun_out/g9/walk.log
[ $rc -eq 0 ] || exit $rc
GCK_LIBRARY=$PWD/gochugaru_amd/libgck_debug.so GCK_DEBUG_PHASES=1 timeout -k 10 200 python -u -m pytest $T -x -v -s \
  --timeout 150 --timeout-method thread > gpurun_out/g9/phases.log 2>&1
echo "phases rc=$?"
grep -o "chain[0-9]*=[^ ]*" gpurun_out/g9/phases.log | sort | uniq | head -20
