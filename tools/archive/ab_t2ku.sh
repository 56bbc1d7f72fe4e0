#!/bin/bash
# DQN update A/B (eager updates, 3 rounds): T2's W3 sums over the present tiles with 8 (ku8)
# or 16 (ku16) independent loads per thread and round
set -u
for rep in 1 2 3; do
  for v in ku8 ku16; do
    timeout -k 10 120 python3 tools/diag/update_forms.py --forms eager --lib shippingenv_amd/_lib/abl/$v.so || exit $?
  done
done
