#!/bin/bash
# round 5: step-kernel grid size at 2^20 (SHIPENV_STEP_BLOCKS: workgroups cap, default 32768 -> 1024
# workgroups of one group per thread; 512 -> two groups per thread), configs 3 and 4, alternating
set -u
O=gpurun_out/${1:-r05w2}; mkdir -p $O
L=shippingenv_amd/_lib/libshipenv_hip.so
for rep in 1 2 3; do
  for b in 0 512 768 256; do
    for c in 3 4; do
      if [ $b = 0 ]; then
        timeout -k 10 60 tools/stepbench --config $c --preroll 1000 --warm 5 --steps 200 $L | sed "s/^{/{\"blocks\": $b, /" >> $O/grid.jsonl || exit 1
      else
        SHIPENV_STEP_BLOCKS=$b timeout -k 10 60 tools/stepbench --config $c --preroll 1000 --warm 5 --steps 200 $L | sed "s/^{/{\"blocks\": $b, /" >> $O/grid.jsonl || exit 1
      fi
    done
  done
done
echo done
