#!/bin/bash
# DQN update A/B (eager updates, 3 rounds): T1's sampler key and ring size passed from the host
# (default) or read on the device (--device-key)
set -u
for rep in 1 2 3; do
  timeout -k 10 120 python3 tools/diag/update_forms.py --forms eager --device-key || exit $?
  timeout -k 10 120 python3 tools/diag/update_forms.py --forms eager || exit $?
done
