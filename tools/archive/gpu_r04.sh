#!/bin/bash
# round-4 GPU pass: the GPU suite, smoke(), the driver's bench command, and the 2-rank launch
# rehearsal (bench.py --gpus 2 spawning its own ranks, both on GPU 0 over gloo)
set -u
TAG=${1:-r04a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $OUT/tests_gpu.log 2>&1 || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_drv.json 2> $OUT/bench_drv.err || exit $?
SHIPENV_REHEARSE=1 timeout -k 10 400 python3 bench.py --gpus 2 --steps 20 --warmup 5 --large-n 0 --no-cpu \
    > $OUT/bench_2rank_rehearsal.json 2> $OUT/bench_2rank_rehearsal.err || exit $?
