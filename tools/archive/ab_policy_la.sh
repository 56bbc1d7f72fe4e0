#!/bin/bash
# bf16 policy kernel A/B (3 rounds, alternating): fc2 fragments read as needed (L0) or
# SHIPENV_POLICY_LOOKAHEAD = 1 / 3 k-steps ahead of their MFMA
set -u
OUT=${1:-gpurun_out/ab_policy_la}
mkdir -p $OUT
for rep in 1 2 3; do
  for L in 0 1 3; do
    timeout -k 10 120 python3 tools/time_policy.py --launches 50 --lib shippingenv_amd/_lib/ab/lib_pol_L$L.so >> $OUT/ab.jsonl || exit $?
  done
done
