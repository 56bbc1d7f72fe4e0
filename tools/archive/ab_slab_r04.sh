#!/bin/bash
# round 4: config 4 (steady state) with the statistics slab as a plain read-modify-write (rmw, the
# product) against the no-return f64 atomics (atomic) and the timing-only build without the done
# list (nodone): N = 2^24 and 2^20, five rounds alternating (tools/stepbench)
set -u
for rep in 1 2 3 4 5; do
  for lib in rmw atomic nodone; do
    timeout -k 10 90 tools/stepbench --config 4 --n 16777216 --preroll 1000 --warm 5 --steps 100 shippingenv_amd/_lib/abl/$lib.so || exit $?
    timeout -k 10 60 tools/stepbench --config 4 --preroll 1000 --warm 5 --steps 200 shippingenv_amd/_lib/abl/$lib.so || exit $?
  done
done
