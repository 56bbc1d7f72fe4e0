#!/bin/bash
# round 4: eager update A/B over shippingenv_amd/_lib/abu (cache-bit and issue-priority variants of T1),
# four rounds alternating (SHIPENV_QT_AUX 16 / 17 / 18 / 2; SHIPENV_QT_PRIO 1 / 2 / 3)
set -u
OUT=${1:-gpurun_out/ab_aux}
mkdir -p $OUT
for rep in 1 2 3 4; do
  for lib in shippingenv_amd/_lib/abu/*.so; do
    timeout -k 10 120 python3 tools/diag/update_forms.py --forms eager --lib $lib >> $OUT/ab_update.jsonl || exit $?
  done
done
