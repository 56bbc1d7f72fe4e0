#!/bin/bash
# N = 2^24: software pipelining (SHIPENV_PREFETCH=1 build) at 2, 4 and 8 groups per thread
# (SHIPENV_STEP_BLOCKS caps) against the product (one group per thread); two rounds.
set -u
set -o pipefail
for rep in 1 2; do
  for cap in 32768 8192 4096 2048; do
    for lib in shippingenv_amd/_lib/abl/a_base.so shippingenv_amd/_lib/abl/p_pref.so; do
      SHIPENV_STEP_BLOCKS=$cap timeout -k 10 90 tools/stepbench --config 3 --n 16777216 --warm 5 --steps 100 $lib | sed "s/^{/{\"cap\": $cap, /" || exit $?
    done
  done
done
