#!/bin/bash
# Time every library under shippingenv_amd/_lib/abl at N=2^20 (configs 3 and 4), alternating libs.
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in shippingenv_amd/_lib/abl/*.so; do
    for c in ${CONFIGS:-3 4}; do
      timeout -k 10 120 python3 tools/time_step.py --lib "$lib" --config $c --steps 300 >> gpurun_out/abl.jsonl || exit $?
    done
  done
done
