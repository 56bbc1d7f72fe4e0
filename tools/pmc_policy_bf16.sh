#!/bin/bash
# SQ counters of the bf16 policy kernel (tools/time_policy.py, 2^20 envs): the stall / wait
# and co-execution counters beside the instruction counts of gpu_final.sh's pass
set -u
OUT=gpurun_out/${1:-pmc_bf16}
mkdir -p $OUT
R=$(pwd)
(export TMPDIR=/tmp && cd /tmp &&
 timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
   --output-format csv -d "$R/$OUT" -o pmc_polb -- python3 "$R/tools/time_policy.py" --preroll 300 --launches 3 > "$R/$OUT/pmc_polb.log" 2>&1 &&
 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC \
   --output-format csv -d "$R/$OUT" -o pmc_polc -- python3 "$R/tools/time_policy.py" --preroll 300 --launches 3 > "$R/$OUT/pmc_polc.log" 2>&1) || exit $?
echo pmc-bf16-ok
