#!/bin/bash
# Build library variants for an A/B timing run (in this container), one per
# "name:-DFLAG=V ..." word of VARIANTS, into shippingenv_amd/_lib/abl/<name>.so:
#   VARIANTS="old:-DSHIPENV_POLICY_EPI=0 new:" bash tools/build_variants.sh
set -eu
D=shippingenv_amd/_lib/abl
mkdir -p $D && rm -f $D/*.so
B="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math --offload-arch=gfx950"
S="shippingenv_amd/csrc/shipenv.hip shippingenv_amd/csrc/mapload.cpp"
for v in ${VARIANTS}; do
  $B ${v#*:} -o $D/${v%%:*}.so $S &
done
wait
ls $D
