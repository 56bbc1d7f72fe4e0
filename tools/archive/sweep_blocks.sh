#!/bin/bash
# Sweep the step kernel's workgroup cap (SHIPENV_STEP_BLOCKS): N=2^20 (configs 3, 4) and 2^24.
set -u
mkdir -p gpurun_out
for b in ${BLOCKS:-256 512 768 1024 2048}; do
  for run in "1048576 3" "1048576 4" "16777216 3"; do
    set -- $run
    SHIPENV_STEP_BLOCKS=$b timeout -k 10 120 python3 tools/time_step.py --n $1 --config $2 --steps 200 | sed "s/^{/{\"blocks\": $b, /" >> gpurun_out/sweep.jsonl || exit $?
  done
done
