#!/bin/bash
# A/B step timing (tools/stepbench) of every build under shippingenv_amd/_lib/abl at the
# driver's short run, the steady state, config 4 and N = 2^24; two rounds, alternating.
set -u
for rep in 1 2; do
  for lib in shippingenv_amd/_lib/abl/*.so; do
    timeout -k 10 60 tools/stepbench --config 3 --warm 5 --steps 20 $lib || exit $?
    timeout -k 10 60 tools/stepbench --config 3 --warm 50 --steps 1000 $lib || exit $?
    timeout -k 10 60 tools/stepbench --config 4 --warm 50 --steps 1000 $lib || exit $?
    timeout -k 10 90 tools/stepbench --config 3 --n 16777216 --warm 5 --steps 100 $lib || exit $?
  done
done
