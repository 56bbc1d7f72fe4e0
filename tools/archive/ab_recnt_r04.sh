#!/bin/bash
# round 4: config 4 at 2^24 / 2^20 (steady state, tools/stepbench): done-list records as plain
# (rmw, the product) or nontemporal (recnt) stores, and without record stores (norecs); five rounds
set -u
for rep in 1 2 3 4 5; do
  for lib in rmw recnt norecs; do
    timeout -k 10 90 tools/stepbench --config 4 --n 16777216 --preroll 1000 --warm 5 --steps 100 shippingenv_amd/_lib/abl/$lib.so || exit $?
    timeout -k 10 60 tools/stepbench --config 4 --preroll 1000 --warm 5 --steps 200 shippingenv_amd/_lib/abl/$lib.so || exit $?
  done
done
