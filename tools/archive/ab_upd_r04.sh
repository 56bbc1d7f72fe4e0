#!/bin/bash
# round 4: eager DQN update A/B over shippingenv_amd/_lib/abp (update_forms.py), four rounds alternating
set -u
OUT=${1:-gpurun_out/ab_upd}
mkdir -p $OUT
for rep in 1 2 3 4; do
  for lib in shippingenv_amd/_lib/abp/*.so; do
    timeout -k 10 120 python3 tools/diag/update_forms.py --forms eager --lib $lib >> $OUT/ab_update.jsonl || exit $?
  done
done
