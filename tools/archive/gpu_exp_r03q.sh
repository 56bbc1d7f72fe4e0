#!/bin/bash
# large_n in steady state beside from reset: the driver's bench command and its kernel trace
set -u
OUT=gpurun_out/r03q
mkdir -p $OUT
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_drv.json 2> $OUT/bench_drv.err || exit $?
bash tools/trace_driver.sh r03q || exit $?
