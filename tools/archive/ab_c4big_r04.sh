#!/bin/bash
# round 4: config 4 (64 ports, auto-reset) in steady state at N = 2^24 and 2^20, builds under
# shippingenv_amd/_lib/abl (tools/stepbench, 1000-step pre-roll), three rounds alternating;
# the PREFETCH builds also at SHIPENV_STEP_BLOCKS=8192 (two groups per thread at 2^24)
set -u
for rep in 1 2 3; do
  for lib in shippingenv_amd/_lib/abl/*.so; do
    timeout -k 10 90 tools/stepbench --config 4 --n 16777216 --preroll 1000 --warm 5 --steps 100 $lib || exit $?
    timeout -k 10 60 tools/stepbench --config 4 --preroll 1000 --warm 5 --steps 200 $lib || exit $?
    case $lib in *pref*|*base*)
      SHIPENV_STEP_BLOCKS=8192 timeout -k 10 90 tools/stepbench --config 4 --n 16777216 --preroll 1000 --warm 5 --steps 100 $lib || exit $?
      SHIPENV_STEP_BLOCKS=8192 timeout -k 10 90 tools/stepbench --config 3 --n 16777216 --preroll 1000 --warm 5 --steps 100 $lib || exit $?
    esac
    timeout -k 10 90 tools/stepbench --config 3 --n 16777216 --preroll 1000 --warm 5 --steps 100 $lib || exit $?
  done
done
