# The dispatch span of k_closure_join (config 4, device batches one at a time) under rocprofv3's
# kernel trace, through HIP and through the engine's HSA queues with each fence / kernarg variant
# (GCK_DEBUG_AQL_FENCE, GCK_DEBUG_AQL_HOSTARGS): attributes the AQL path's extra microseconds.
# (the switches act in the debug build only: make -C gochugaru_amd/csrc DEBUG=1)
#   bash tools/aql_span.sh <out dir> [tags]   (on the GPU box, from the repo root; tags: the variants to run)
set -e
OUT=$1
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ONLY=" ${*:2} "
run() {
  local tag=$1
  shift
  if [ "$ONLY" != "  " ] && [[ "$ONLY" != *" $tag "* ]]; then return 0; fi
  env GCK_LIBRARY=$PWD/gochugaru_amd/libgck_debug.so "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/$tag" -o kt --output-format csv -- \
    python3 tools/host_probe.py --phases device --lone 40 --batches 40 > "$OUT/$tag.json" 2> "$OUT/$tag.err"
  python3 - "$OUT/$tag" "$tag" <<'PY'
import csv, sys, numpy as np
rows = [r for r in csv.DictReader(open(sys.argv[1] + "/kt_kernel_trace.csv")) if "closure_join" in r["Kernel_Name"]]
d = np.array([int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]) / 1e3
print(f"{sys.argv[2]}: n={len(d)} lone median {np.median(d[16:59]):.2f} us, min {d[16:59].min():.2f}")
PY
  find "$OUT/$tag" -name "*kernel_trace.csv" -delete
}
run hip GCK_AQL=0
run aql_default GCK_AQL=1
run aql_acq0_rel2 GCK_DEBUG_AQL_FENCE=0,2
run aql_acq1_rel1 GCK_DEBUG_AQL_FENCE=1,1
run aql_acq2_rel2 GCK_DEBUG_AQL_FENCE=2,2
run aql_acq0_rel1 GCK_DEBUG_AQL_FENCE=0,1
run aql_hostargs GCK_DEBUG_AQL_HOSTARGS=1
run aql_noprof GCK_DEBUG_AQL_NOPROF=1
run aql_single GCK_DEBUG_AQL_SINGLE=1
run aql_signal GCK_DEBUG_AQL_SIGNAL=1
run hip_selfpub GCK_AQL=0 GCK_DEBUG_HIP_SELFPUB=1
GCK_DEBUG_AQL=1 timeout -k 10 200 python3 tools/host_probe.py --phases device --lone 5 --batches 10 2>&1 | grep "gck aql\] k_closure" | head -3
