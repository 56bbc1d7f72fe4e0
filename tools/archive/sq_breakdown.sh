#!/bin/bash
# Wave-time decomposition of the step kernel (config 3, N=2^20): WAIT_ANY (parked on
# s_waitcnt / barrier) + WAIT_INST_ANY (issue stall) + ACTIVE_INST_ANY ~= WAVE_CYCLES.
# Usage: bash tools/sq_breakdown.sh [lib.so] [tag]   (GPU box; one counter pass per line)
set -u
R=$(pwd); LIB=${1:-$R/shippingenv_amd/_lib/libshipenv_hip.so}; TAG=${2:-cur}
OUT=$R/gpurun_out/sqb_$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_WAVES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM"
i=0
for p in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $p --output-format csv -d "$OUT/p$i" -o sq -- python3 $R/tools/time_step.py --lib $LIB --steps 20 > "$OUT/p$i.log" 2>&1 || exit $?
done
