#!/bin/bash
# r04: config 5 and the driver-sized headline again (box-to-box spread).
set -o pipefail
out=gpurun_out/j43
mkdir -p $out
for r in 1 2; do
timeout -k 10 300 python -u bench.py --config mixed --steps 20 --warmup 5 --no-cpu > $out/mixed_$r.json 2> $out/mixed_$r.err || exit 2
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > $out/driver_$r.json 2> $out/driver_$r.err || exit 3
done
