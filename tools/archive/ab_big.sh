#!/bin/bash
# N = 2^24 floors: the product, the no-logic build (ABLATE=1), no staging either (ABLATE=2),
# with the product's loads (temporal at this N) and forced nontemporal loads
set -u
set -o pipefail
for rep in 1 2; do
  for lib in shippingenv_amd/_lib/abl/*.so; do
    timeout -k 10 90 tools/stepbench --config 3 --n 16777216 --warm 5 --steps 100 $lib | sed 's/^{/{"ntl": 0, /' || exit $?
    SHIPENV_NT_LOADS=1 timeout -k 10 90 tools/stepbench --config 3 --n 16777216 --warm 5 --steps 100 $lib | sed 's/^{/{"ntl": 1, /' || exit $?
  done
done
