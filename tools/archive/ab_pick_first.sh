#!/bin/bash
# DQN update A/B (eager updates, 3 rounds, alternating): the previous build against T1 issuing
# the pick's loads ahead of the fragment loads, waves 1-7 waiting 0 / 8 / 16 x 64 cycles
set -u
OUT=${1:-gpurun_out/ab_pick_first}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dqn.py -m gpu > $OUT/test_gpu_dqn.log 2>&1 || exit $?
for rep in 1 2 3; do
  for lib in prev sleep0 sleep8 sleep16; do
    timeout -k 10 120 python3 tools/diag/update_forms.py --forms eager --lib shippingenv_amd/_lib/ab/lib_$lib.so >> $OUT/ab.jsonl || exit $?
  done
done
