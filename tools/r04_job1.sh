# round-4 GPU job: the partitioned tests not yet confirmed, the Watch tests (delta, nested churn,
# concurrent checks), a small partitioned bench line. Each step has its own time limit.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04e
timeout -k 10 700 python -u -m pytest tests/test_gpu_partition.py -k "fraction or rccl or config4 or watch" -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r04e/part.log 2>&1 || { tail -30 gpurun_out/r04e/part.log; exit 1; }
tail -2 gpurun_out/r04e/part.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_delta.py tests/test_gpu_watch_concurrent.py tests/test_gpu_watch_nested.py -x -q -s --timeout 600 --timeout-method thread > gpurun_out/r04e/watch.log 2>&1 || { tail -30 gpurun_out/r04e/watch.log; exit 1; }
tail -2 gpurun_out/r04e/watch.log
grep -h "worst_check_ms\|apply_s" gpurun_out/r04e/watch.log | tail -5
timeout -k 10 300 python3 bench.py --partitioned --tuples 1e7 --steps 20 --warmup 3 > gpurun_out/r04e/part_bench.json 2> gpurun_out/r04e/part_bench.err || { tail -20 gpurun_out/r04e/part_bench.err; exit 1; }
tail -c 800 gpurun_out/r04e/part_bench.json
