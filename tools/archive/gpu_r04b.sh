#!/bin/bash
# round 4: step_seq mark test, the driver's bench command, config-4 2^24 A/B
set -u
OUT=gpurun_out/${1:-r04b}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k step_seq > $OUT/tests_seq.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --large-n 0 --no-cpu --train-steps 0 --rollouts 0 > $OUT/bench_drv.json 2> $OUT/bench_drv.err || exit $?
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --large-n 0 --no-cpu --train-steps 0 --rollouts 0 > $OUT/bench_drv2.json 2> $OUT/bench_drv2.err || exit $?
timeout -k 10 900 bash tools/ab_c4big_r04.sh > $OUT/ab_c4big.jsonl 2> $OUT/ab_c4big.err || exit $?
