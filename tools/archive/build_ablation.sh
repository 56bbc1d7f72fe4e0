#!/bin/bash
# Build the timing-only variants tools/ablate_libs.sh compares (in this container):
#   cur.so     the product build
#   ablate.so  SHIPENV_ABLATE=1: the same memory traffic with no logic and no draws
# Extra -D variants: EXTRA="name:-DFLAG=1 name2:-DFLAG2" (e.g. the Philox round count).
set -eu
D=shippingenv_amd/_lib/abl
mkdir -p $D && rm -f $D/*.so
B="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math --offload-arch=gfx950"
S="shippingenv_amd/csrc/shipenv.hip shippingenv_amd/csrc/mapload.cpp"
$B -o $D/cur.so $S
$B -DSHIPENV_ABLATE=1 -o $D/ablate.so $S
for v in ${EXTRA:-}; do
  $B ${v#*:} -o $D/${v%%:*}.so $S
done
ls $D
