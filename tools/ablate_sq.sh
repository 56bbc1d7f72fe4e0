#!/bin/bash
# SQ instruction counts of each ablation build (config 3, N=2^20, 10 steps after 200 warm steps).
set -u
R=$(pwd); OUT=$R/gpurun_out/ablate_sq; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
for lib in $R/shippingenv_amd/_lib/ablate/*.so; do
  name=$(basename $lib .so)
  timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$OUT/$name" -o sq -- python3 $R/tools/time_step.py --lib $lib --steps 20 > "$OUT/$name.log" 2>&1 || exit $?
done
