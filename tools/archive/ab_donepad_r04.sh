#!/bin/bash
# round 4: config 4 at N = 2^24 and 2^20 (steady state, tools/stepbench): the done list's records
# padded to 128-B lines (pad8, the product), 64-B (pad4), not padded (pad1), and the timing-only
# build without record stores (norecs); five rounds alternating
set -u
for rep in 1 2 3 4 5; do
  for lib in pad8 pad1 pad4 norecs; do
    timeout -k 10 90 tools/stepbench --config 4 --n 16777216 --preroll 1000 --warm 5 --steps 100 shippingenv_amd/_lib/abl/$lib.so || exit $?
    timeout -k 10 60 tools/stepbench --config 4 --preroll 1000 --warm 5 --steps 200 shippingenv_amd/_lib/abl/$lib.so || exit $?
  done
done
