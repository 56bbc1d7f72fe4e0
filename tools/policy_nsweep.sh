#!/bin/bash
# policy time against N (tiles per wave 1..16 at 2^17..2^21): the per-tile slope and the
# fixed cost (network / world staging, launch) of se_policy and se_policy_f32
set -u
for prec in ${PRECS:-bf16 f32}; do
  for lg in 13 15 17 18 19 20 21; do
    timeout -k 10 120 python tools/time_policy.py --precision $prec --launches 40 --n $((1 << lg)) || exit 1
  done
done
exit 0
