cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g8
T=tests/test_gpu_labels.py::test_direct_grant_churn_keeps_the_tables
GCK_LIBRARY=$PWD/_ab/gochugaru_amd/libgck.so timeout -k 10 200 python -u -m pytest $T -x -v --timeout 150 \
  --timeout-method thread > gpurun_out/g8/old.log 2>&1
rc=$?
echo "old rc=$rc"; tail -3 gpurun_out/g8/old.log
[ $rc -eq 0 ] || exit $rc
GCK_LIBRARY=$PWD/gochugaru_amd/libgck_walkdbg.so timeout -k 10 200 python -u -m pytest $T -x -v -s --timeout 150 \
  --timeout-method thread > gpurun_out/g8/walk.log 2>&1
rc=$?
echo "walkdbg rc=$rc"; tail -3 gpurun_out/g8/walk.log; grep -c "^walk" gpurun_out/g8/walk.log
exit $rc
