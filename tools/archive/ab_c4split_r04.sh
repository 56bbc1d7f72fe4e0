#!/bin/bash
# round 4: where config 4's time goes at N = 2^24 (steady state, tools/stepbench): configs 3 / 4 /
# 5 (64 ports, no auto-reset) / 6 (5 ports, auto-reset) on the product build, then config 4 on
# the SHIPENV_ABL4 timing-only builds (no done list, no stats, neither); three rounds
set -u
for rep in 1 2 3; do
  for c in 3 4 5 6; do
    timeout -k 10 90 tools/stepbench --config $c --n 16777216 --preroll 1000 --warm 5 --steps 100 shippingenv_amd/_lib/abl/base.so || exit $?
  done
  for lib in nodone nostats neither; do
    timeout -k 10 90 tools/stepbench --config 4 --n 16777216 --preroll 1000 --warm 5 --steps 100 shippingenv_amd/_lib/abl/$lib.so || exit $?
  done
done
