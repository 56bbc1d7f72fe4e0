#!/bin/bash
# round 5: the DQN update (T1 + T2) over the library builds under shippingenv_amd/_lib/ablu,
# ROUNDS rounds alternating (tools/time_train.py --eager, 2^20 envs, B = 8192); one JSON line per run
set -u
for rep in $(seq 1 ${ROUNDS:-3}); do
  for lib in ${LIBS:-shippingenv_amd/_lib/ablu/*.so}; do
    echo "{\"lib\": \"$lib\", \"rep\": $rep}"
    timeout -k 10 120 python tools/time_train.py --eager --iters 40 --lib $lib || exit 1
  done
done
exit 0
