#!/bin/bash
set -u
OUT=gpurun_out/r03z
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dqn.py -m gpu > $OUT/test_dqn.log 2>&1 || exit $?
bash tools/ab_t1split.sh > $OUT/ab_t1split.jsonl 2> $OUT/ab_t1split.err || exit $?
