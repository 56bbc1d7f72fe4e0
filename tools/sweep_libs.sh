#!/bin/bash
# Time each library under shippingenv_amd/_lib/ablate at several workgroup caps:
# N=2^20 configs 3 and 4, and N=2^24 config 3 (GPU box). BLOCKS overrides the caps.
set -u
mkdir -p gpurun_out
for lib in shippingenv_amd/_lib/ablate/*.so; do
  for b in ${BLOCKS:-256 512 2048}; do
    for run in "1048576 3" "1048576 4" "16777216 3"; do
      set -- $run
      SHIPENV_STEP_BLOCKS=$b timeout -k 10 120 python3 tools/time_step.py --lib $lib --n $1 --config $2 --steps 200 | sed "s/^{/{\"blocks\": $b, /" >> gpurun_out/sweep_libs.jsonl || exit $?
    done
  done
done
