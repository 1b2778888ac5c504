set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
i=0
for ctrs in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum" "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCP_LATENCY_sum TCP_TA_TCP_STATE_READ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctrs -d gpurun_out/pmc/p$i -o p$i --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/pmc/p$i.json 2> gpurun_out/pmc/p$i.err
done
