#!/bin/bash
# Build library variants for an A/B timing run (in this container), one per
# "name:-DFLAG=V,-DFLAG2=W" word of VARIANTS (flags separated by commas), into
# shippingenv_amd/_lib/abl/<name>.so:
#   VARIANTS="a:-DSHIPENV_FC2_SPLIT=2 b:-DSHIPENV_FC2_SPLIT=4,-DSHIPENV_POLICY_BLOCK=640" bash tools/build_variants.sh
set -eu
D=${ABL_DIR:-shippingenv_amd/_lib/abl}
mkdir -p $D && rm -f $D/*.so
B="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math --offload-arch=gfx950"
S="shippingenv_amd/csrc/shipenv.hip shippingenv_amd/csrc/mapload.cpp"
for v in ${VARIANTS}; do
  f=${v#*:}
  $B ${f//,/ } -o $D/${v%%:*}.so $S &
done
wait
ls $D
