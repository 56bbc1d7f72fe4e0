#!/bin/bash
# the bf16 or f32 (split-bf16) policy over the library builds under shippingenv_amd/_lib/abl,
# ROUNDS rounds alternating (tools/time_policy.py, 2^20 envs); one JSON line per run
set -u
for rep in $(seq 1 ${ROUNDS:-3}); do
  for lib in ${LIBS:-shippingenv_amd/_lib/abl/*.so}; do
    timeout -k 10 120 python tools/time_policy.py --precision ${PREC:-f32} --launches 20 --preroll ${PREROLL:-0} --lib $lib || exit 1
  done
done
exit 0
