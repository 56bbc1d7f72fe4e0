#!/bin/bash
# Step kernel wall time at N = 2^20, 2^22, 2^24 (config 3) and 2^20 (config 4).
set -u
LIB=${LIB:-shippingenv_amd/_lib/libshipenv_hip.so}
for run in 1048576:3 1048576:4 4194304:3 16777216:3; do
  n=${run%%:*}; c=${run##*:}
  timeout -k 10 120 python3 tools/time_step.py --lib $LIB --n $n --config $c --steps 200 >> gpurun_out/sizes.jsonl || exit $?
done
