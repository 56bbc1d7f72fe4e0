#!/bin/bash
# SQ instruction-mix counters for the step kernel (config 3, N=2^20), one pass per group.
set -u
TAG=${1:-sq}
R=$(pwd)
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
PY="python3 $R/tools/prof_step.py"
cd /tmp
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM --output-format csv -d "$OUT" -o sq_a -- $PY --config 3 --steps 10 > "$OUT/a.log" 2>&1 &&
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F64 SQ_WAVES --output-format csv -d "$OUT" -o sq_b -- $PY --config 3 --steps 10 > "$OUT/b.log" 2>&1 &&
timeout -k 10 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVES --output-format csv -d "$OUT" -o sq_c -- $PY --config 3 --steps 10 > "$OUT/c.log" 2>&1 &&
timeout -k 10 200 rocprofv3 --pmc SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE SQ_WAVES --output-format csv -d "$OUT" -o sq_d -- $PY --config 3 --steps 10 > "$OUT/d.log" 2>&1
