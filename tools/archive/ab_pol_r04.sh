#!/bin/bash
# round 4: bf16 policy launch A/B (tools/time_policy.py, 2^20 envs) over shippingenv_amd/_lib/abp, five rounds alternating
set -u
OUT=${1:-gpurun_out/ab_pol}
mkdir -p $OUT
for rep in 1 2 3 4 5; do
  for lib in shippingenv_amd/_lib/abp/*.so; do
    timeout -k 10 120 python3 tools/time_policy.py --launches 50 --lib $lib >> $OUT/ab_policy.jsonl || exit $?
  done
done
