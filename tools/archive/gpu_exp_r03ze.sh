#!/bin/bash
set -u
OUT=gpurun_out/r03ze
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dqn.py -m gpu > $OUT/test_dqn.log 2>&1 || exit $?
bash tools/ab_hostkey.sh > $OUT/ab.jsonl 2> $OUT/ab.err || exit $?
bash tools/ab_w1merge.sh > $OUT/ab_w1.jsonl 2> $OUT/ab_w1.err || exit $?
