#!/bin/bash
# round 4: wave issue priority (s_setprio) A/B: the bf16 policy over shippingenv_amd/_lib/abp
# (tools/time_policy.py) and the eager update over shippingenv_amd/_lib/abu, alternating builds
set -u
OUT=${1:-gpurun_out/ab_prio}
mkdir -p $OUT
for rep in 1 2 3 4; do
  for lib in shippingenv_amd/_lib/abp/*.so; do
    timeout -k 10 120 python3 tools/time_policy.py --launches 50 --lib $lib >> $OUT/ab_policy.jsonl || exit $?
  done
  for lib in shippingenv_amd/_lib/abu/*.so; do
    timeout -k 10 120 python3 tools/diag/update_forms.py --forms eager --lib $lib >> $OUT/ab_update.jsonl || exit $?
  done
done
