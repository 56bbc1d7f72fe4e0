#!/bin/bash
# DQN update A/B (eager updates, 3 rounds, alternating): the previous build (one accumulation
# chain per MFMA tile) against the working tree's (two chains: even / odd k-steps; dW2's
# column tiles in pairs), then the working tree's phase stamps
set -u
OUT=${1:-gpurun_out/ab_chains}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dqn.py -m gpu > $OUT/test_gpu_dqn.log 2>&1 || exit $?
for rep in 1 2 3; do
  timeout -k 10 120 python3 tools/diag/update_forms.py --forms eager --lib shippingenv_amd/_lib/ab/lib_prev.so >> $OUT/ab.jsonl || exit $?
  timeout -k 10 120 python3 tools/diag/update_forms.py --forms eager >> $OUT/ab.jsonl || exit $?
done
bash tools/qtrace_ab.sh $OUT
