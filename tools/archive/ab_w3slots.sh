#!/bin/bash
# DQN update A/B (eager updates, 3 rounds, alternating): the HEAD library (action-tile dW3
# partials) against the working tree's (dW3 over each tile's distinct actions, W3 row blocks)
set -u
OUT=${1:-gpurun_out/ab_w3slots}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dqn.py -m gpu > $OUT/test_gpu_dqn.log 2>&1 || exit $?
for rep in 1 2 3; do
  timeout -k 10 120 python3 tools/diag/update_forms.py --forms eager --lib shippingenv_amd/_lib/ab/lib_head.so >> $OUT/ab.jsonl || exit $?
  timeout -k 10 120 python3 tools/diag/update_forms.py --forms eager >> $OUT/ab.jsonl || exit $?
done
