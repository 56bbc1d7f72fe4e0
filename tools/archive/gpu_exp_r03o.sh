#!/bin/bash
# round-3 checkpoint: the GPU suite, the driver's bench command twice, and its kernel trace
set -u
OUT=gpurun_out/r03o
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > $OUT/tests_gpu.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_drv.json 2> $OUT/bench_drv.err || exit $?
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_drv2.json 2> $OUT/bench_drv2.err || exit $?
bash tools/trace_driver.sh r03o || exit $?
