#!/bin/bash
# Sweep the step kernel's workgroup cap x software pipelining (SHIPENV_STEP_PIPE) at
# N=2^20 (configs 3, 4) and 2^24 (config 3). GPU box; one JSON line per point.
set -u
mkdir -p gpurun_out
for pipe in ${PIPES:-0 1}; do
  for b in ${BLOCKS:-1024 512 256 128}; do
    for run in ${RUNS:-"1048576:3" "1048576:4" "16777216:3"}; do
      n=${run%%:*}; c=${run##*:}
      SHIPENV_STEP_PIPE=$pipe SHIPENV_STEP_BLOCKS=$b timeout -k 10 120 python3 tools/time_step.py --n $n --config $c --steps 200 \
        | sed "s/^{/{\"pipe\": $pipe, \"blocks\": $b, /" >> gpurun_out/sweep_pipe.jsonl || exit $?
    done
  done
done
