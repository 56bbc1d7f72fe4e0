#!/bin/bash
# bf16 policy A/B (3 rounds, alternating): exploration draws one Philox pass per tile (pd0)
# or two tiles per pass (pd1, SHIPENV_POLICY_PAIRED_DRAWS); the policy GPU tests first
set -u
OUT=${1:-gpurun_out/ab_policy_draws}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_policy.py tests/test_gpu_dqn.py -m gpu > $OUT/tests.log 2>&1 || exit $?
for rep in 1 2 3; do
  for P in 0 1; do
    timeout -k 10 120 python3 tools/time_policy.py --launches 50 --lib shippingenv_amd/_lib/ab/lib_pd$P.so >> $OUT/ab.jsonl || exit $?
  done
done
