#!/bin/bash
# round 4: what the world staging costs config 3 at 2^20 (steady state, tools/stepbench): the
# product, the timing-only traffic build (abl1) and the same without staging (abl2); five rounds
set -u
for rep in 1 2 3 4 5; do
  for lib in prod abl1 abl2; do
    timeout -k 10 60 tools/stepbench --config 3 --preroll 1000 --warm 5 --steps 200 shippingenv_amd/_lib/abl/$lib.so || exit $?
  done
done
