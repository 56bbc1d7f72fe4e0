#!/bin/bash
# DQN update A/B (eager updates, 3 rounds): qtnt0 = round-3 T1/T2, qtnt1 = T1's gradient
# partials with nontemporal stores (SHIPENV_QT_NT=1), t2new = T2 with the Adam operands loaded
# ahead of the sums and the W3 sums over the present tiles only (now the tree's T2; qtnt0 /
# qtnt1 were built from the tree before that change, with -DSHIPENV_QT_NT=0 / 1)
set -u
for rep in 1 2 3; do
  for v in qtnt0 qtnt1 t2new; do
    timeout -k 10 120 python3 tools/diag/update_forms.py --forms eager --lib shippingenv_amd/_lib/abl/$v.so || exit $?
  done
done
