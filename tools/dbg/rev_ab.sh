cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g5
for v in orig noinflight nolabels noclosure; do
  timeout -k 10 60 python3 -u tools/dbg/rev_repro.py $v >> gpurun_out/g5/rev.log 2>&1 || echo "$v rc=$?" >> gpurun_out/g5/rev.log
done
GCK_AQL=0 timeout -k 10 60 python3 -u tools/dbg/rev_repro.py orig_noaql >> gpurun_out/g5/rev.log 2>&1 || echo "noaql rc=$?" >> gpurun_out/g5/rev.log
cat gpurun_out/g5/rev.log | grep -v Warning
