#!/bin/bash
# Time every library under shippingenv_amd/_lib/abl (configs 3 and 4 at N=2^20 by
# default; RUNS="n:config ..." overrides), alternating libraries, two rounds.
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in shippingenv_amd/_lib/abl/*.so; do
    for run in ${RUNS:-1048576:3 1048576:4}; do
      n=${run%%:*}; c=${run##*:}
      timeout -k 10 120 python3 tools/time_step.py --lib "$lib" --n $n --config $c --steps 300 >> gpurun_out/abl.jsonl || exit $?
    done
  done
done
