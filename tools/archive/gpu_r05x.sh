#!/bin/bash
# round 5: f32 policy tests on the product library (fc1 bias folded into the split-bf16 fragments),
# then the f32 policy A/B over shippingenv_amd/_lib/ablx (fold on / off, issue priority)
set -u
O=gpurun_out/${1:-r05x2}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_policy.py tests/test_gpu_dqn.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
LIBS="$(ls shippingenv_amd/_lib/ablx/*.so)" PREC=f32 ROUNDS=5 bash tools/ab_policy_r05.sh > $O/ab_policy_f32.jsonl 2>$O/ab.err || { tail $O/ab.err; exit 1; }
echo done
