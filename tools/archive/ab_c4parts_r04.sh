#!/bin/bash
# round 4: config 4 at N = 2^24 and 2^20 (steady state, tools/stepbench) on the product build (rmw)
# and the SHIPENV_ABL4 timing-only builds: no statistics, no done list, the done list without its
# record stores, without its count stores; five rounds alternating
set -u
for rep in 1 2 3 4 5; do
  for lib in rmw nostats nodone norecs nocount; do
    timeout -k 10 90 tools/stepbench --config 4 --n 16777216 --preroll 1000 --warm 5 --steps 100 shippingenv_amd/_lib/abl/$lib.so || exit $?
    timeout -k 10 60 tools/stepbench --config 4 --preroll 1000 --warm 5 --steps 200 shippingenv_amd/_lib/abl/$lib.so || exit $?
  done
done
