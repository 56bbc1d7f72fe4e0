#!/bin/bash
# round 5: DQN tests on the product library, then back-to-back update A/B (tools/time_update.py)
# and training-loop A/B (tools/ab_update_r05.sh) over shippingenv_amd/_lib/ablu, and phase stamps
set -u
O=gpurun_out/${1:-r05v2}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dqn.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2 3; do
  for lib in shippingenv_amd/_lib/ablu/*.so; do
    timeout -k 10 120 python tools/time_update.py --lib $lib >> $O/time_update.jsonl 2>>$O/err.log || { tail $O/err.log; exit 1; }
  done
done
ROUNDS=2 bash tools/ab_update_r05.sh > $O/ab_update.jsonl 2>>$O/err.log || { tail $O/err.log; exit 1; }
for q in shippingenv_amd/_lib/ablq/*.so; do
  echo "{\"lib\": \"$q\"}" >> $O/qtrace.jsonl; timeout -k 10 120 python tools/qtrain_trace.py --lib $q >> $O/qtrace.jsonl 2>>$O/err.log || { tail $O/err.log; exit 1; }
done
echo done
