#!/bin/bash
# DQN update A/B (eager updates, 3 rounds): the tree's library against w1merge (T2's W1 blocks
# reduce their seven sums, sum w and the loss in one block_sum, and pick column sums by selects)
set -u
for rep in 1 2 3; do
  timeout -k 10 120 python3 tools/diag/update_forms.py --forms eager || exit $?
  timeout -k 10 120 python3 tools/diag/update_forms.py --forms eager --lib shippingenv_amd/_lib/abl/w1merge.so || exit $?
done
