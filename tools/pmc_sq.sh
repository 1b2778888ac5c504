# SQ counters of the bundle kernels (instruction mix, waits, LDS), one counter group per pass.
# Usage on the GPU box: bash tools/pmc_sq.sh <out dir under gpurun_out>
set -e
OUT=${1:-gpurun_out/sq}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" \
            "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $ctrs -d "$OUT/p$i" -o p$i --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-oracle --host-steps 0 > "$OUT/p$i.json" 2> "$OUT/p$i.err"
done
