#!/bin/bash
# round 5: config 4 with and without nontemporal state loads (SHIPENV_NT_LOADS) from 2^20 to
# 2^25 (tools/stepbench, the product library, 1000-step pre-roll), ROUNDS rounds alternating.
set -u
L=${LIB:-shippingenv_amd/_lib/libshipenv_hip.so}
for rep in $(seq 1 ${ROUNDS:-2}); do
  for lg in 20 21 22 23 24 25; do
    n=$((1 << lg)); k=$(( lg >= 24 ? 50 : 200 ))
    for nt in 0 1; do
      SHIPENV_NT_LOADS=$nt timeout -k 10 120 tools/stepbench --config ${CONFIG:-4} --n $n --preroll 1000 --warm 5 --steps $k $L \
        | sed "s/^{/{\"nt_loads\": $nt, /" || exit 1
    done
  done
done
exit 0
