#!/bin/bash
# round 4 A/B (3 rounds, alternating) over the builds in shippingenv_amd/_lib/abp: the bf16
# policy launch (tools/time_policy.py, 2^20 envs) and the eager DQN update (update_forms.py)
set -u
OUT=${1:-gpurun_out/ab_pol_upd}
mkdir -p $OUT
for rep in 1 2 3; do
  for lib in shippingenv_amd/_lib/abp/*.so; do
    timeout -k 10 120 python3 tools/time_policy.py --launches 50 --lib $lib >> $OUT/ab_policy.jsonl || exit $?
    timeout -k 10 120 python3 tools/diag/update_forms.py --forms eager --lib $lib >> $OUT/ab_update.jsonl || exit $?
  done
done
