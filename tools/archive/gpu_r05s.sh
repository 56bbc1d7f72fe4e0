#!/bin/bash
# round 5: DQN + policy GPU tests on the product library (split-bf16 T1 forward), the update
# A/B (f32 / x3 / x3 unfenced) and the bf16 policy A/B (round-4 epilogue / masked -inf)
set -u
O=gpurun_out/${1:-r05s}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dqn.py tests/test_gpu_policy.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
ROUNDS=3 bash tools/ab_update_r05.sh > $O/ab_update.jsonl 2>$O/ab.err || { tail $O/ab.err; exit 1; }
LIBS="shippingenv_amd/_lib/abl/a_bf16old.so shippingenv_amd/_lib/abl/b_bf16mask.so" PREC=bf16 ROUNDS=3 bash tools/ab_policy_r05.sh > $O/ab_policy_bf16.jsonl 2>>$O/ab.err || { tail $O/ab.err; exit 1; }
echo done
