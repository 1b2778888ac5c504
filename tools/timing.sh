set -e
mkdir -p gpurun_out/sw
touch gochugaru_amd/csrc/bundle.inc && make -C gochugaru_amd/csrc TIMING=1 > /dev/null
rm -f gpurun_out/sw/t.bin
GCK_DEBUG_TIMING=gpurun_out/sw/t timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu "$@" > gpurun_out/sw/t.json 2> gpurun_out/sw/t.err
python tests/analyze_timing.py gpurun_out/sw/t.bin > gpurun_out/sw/t.txt
