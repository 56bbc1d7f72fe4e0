#!/bin/bash
# Sweep the step kernel's workgroup cap (SHIPENV_STEP_BLOCKS) at N=2^20 and 2^24.
set -u
mkdir -p gpurun_out
for b in 256 512 768 1024 2048; do
  for n in 1048576 16777216; do
    SHIPENV_STEP_BLOCKS=$b timeout -k 10 120 python3 tools/time_step.py --n $n --steps 200 | sed "s/^{/{\"blocks\": $b, /" >> gpurun_out/sweep.jsonl || exit $?
  done
done
