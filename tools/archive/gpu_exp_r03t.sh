#!/bin/bash
# update drawing its own minibatch: DQN tests, the update forms, the training leg
set -u
OUT=gpurun_out/r03t
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dqn.py -m gpu > $OUT/test_dqn.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/diag/update_forms.py > $OUT/update_forms.jsonl 2> $OUT/update_forms.err || exit $?
timeout -k 10 300 python3 tools/time_train.py --iters 50 > $OUT/time_train.jsonl 2> $OUT/time_train.err || exit $?
