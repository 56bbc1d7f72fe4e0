#!/bin/bash
# step workgroup size A/B (tools/stepbench, 3 rounds, alternating) of the builds under
# shippingenv_amd/_lib/abl: N = 2^24 and 2^20 after 1000 warm steps (steady mix), config 4
set -u
for rep in 1 2 3; do
  for lib in shippingenv_amd/_lib/abl/*.so; do
    timeout -k 10 120 tools/stepbench --config 3 --n 16777216 --warm 1000 --steps 100 $lib || exit $?
    timeout -k 10 60 tools/stepbench --config 3 --warm 1000 --steps 1000 $lib || exit $?
    timeout -k 10 60 tools/stepbench --config 4 --warm 1000 --steps 1000 $lib || exit $?
  done
done
