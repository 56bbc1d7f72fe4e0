#!/bin/bash
# Time every library under shippingenv_amd/_lib/ablate at N=2^20 and 2^24 (GPU box).
set -u
mkdir -p gpurun_out
for lib in shippingenv_amd/_lib/ablate/*.so; do
  for n in 1048576 16777216; do
    timeout -k 10 120 python3 tools/time_step.py --lib "$lib" --n $n --steps 200 >> gpurun_out/ablate.jsonl 2>> gpurun_out/ablate.err || exit $?
  done
done
