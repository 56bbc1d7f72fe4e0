#!/bin/bash
# DQN update A/B (eager updates, 3 rounds): t2new = T1 with one MFMA chain per tile (8 waves),
# t1split = T1 with each tile's K split over two waves (16 waves; measured slower and not kept,
# so that build is not reproducible from the tree: DESIGN.md section 13 describes it)
set -u
for rep in 1 2 3; do
  for v in t2new t1split; do
    timeout -k 10 120 python3 tools/diag/update_forms.py --forms eager --lib shippingenv_amd/_lib/abl/$v.so || exit $?
  done
done
