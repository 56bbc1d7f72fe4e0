#!/bin/bash
set -u
OUT=gpurun_out/r03w
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dqn.py -m gpu > $OUT/test_dqn.log 2>&1 || exit $?
bash tools/ab_qtnt.sh > $OUT/ab_qtnt.jsonl 2> $OUT/ab_qtnt.err || exit $?
