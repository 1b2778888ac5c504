cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g6
for v in x40first single2 sync sleep nomhash; do
  timeout -k 10 60 python3 -u tools/dbg/rev_repro2.py $v 2>&1 | grep -v amdgpu.ids >> gpurun_out/g6/rev.log || echo "$v rc=$?" >> gpurun_out/g6/rev.log
done
cat gpurun_out/g6/rev.log
