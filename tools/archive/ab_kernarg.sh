#!/bin/bash
# HIP_FORCE_DEV_KERNARG=0 / 1 (kernel arguments in host or device memory), alternating: the
# step kernel (config 3 and 4), back-to-back updates, the bf16 policy at config 5's state
set -u
OUT=gpurun_out/${1:-r06ka}
mkdir -p $OUT
for rep in 1 2; do
  for k in 0 1; do
    export HIP_FORCE_DEV_KERNARG=$k
    timeout -k 10 120 python3 tools/time_step.py --config 3 | sed "s/^{/{\"kernarg_dev\": $k, \"what\": \"c3\", /" >> $OUT/ab.jsonl || exit $?
    timeout -k 10 120 python3 tools/time_step.py --config 4 | sed "s/^{/{\"kernarg_dev\": $k, \"what\": \"c4\", /" >> $OUT/ab.jsonl || exit $?
    timeout -k 10 120 python3 tools/time_update.py | sed "s/^{/{\"kernarg_dev\": $k, \"what\": \"update\", /" >> $OUT/ab.jsonl || exit $?
    timeout -k 10 120 python3 tools/time_policy.py --preroll 300 | sed "s/^{/{\"kernarg_dev\": $k, \"what\": \"pol_bf16\", /" >> $OUT/ab.jsonl || exit $?
  done
done
echo ka-ok
