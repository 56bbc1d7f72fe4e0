#!/bin/bash
# round 5: DQN GPU tests on the product library (split-bf16 T1 forward + backward), the update
# A/B (f32 / x3 forward / x3 forward + backward / unfenced) and T1 / T2 phase stamps
set -u
O=gpurun_out/${1:-r05t}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dqn.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
ROUNDS=3 bash tools/ab_update_r05.sh > $O/ab_update.jsonl 2>$O/ab.err || { tail $O/ab.err; exit 1; }
for q in shippingenv_amd/_lib/ablq/*.so; do
  echo "{\"lib\": \"$q\"}" >> $O/qtrace.jsonl; timeout -k 10 120 python tools/qtrain_trace.py --lib $q >> $O/qtrace.jsonl 2>>$O/ab.err || { tail $O/ab.err; exit 1; }
done
echo done
