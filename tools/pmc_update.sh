#!/bin/bash
# SQ counters of the DQN update's kernels (tools/diag/update_forms.py, eager), one pass
set -u
R=$(pwd)
OUT=$R/gpurun_out/${1:-r03x}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES \
    --output-format csv -d "$OUT" -o pmc_upd -- python3 "$R/tools/diag/update_forms.py" --forms eager --iters 10 > "$OUT/pmc_upd.log" 2>&1 || exit $?
# instruction counts of T1 / T2 (back-to-back updates, tools/time_update.py), a second pass
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU \
    --output-format csv -d "$OUT" -o pmc_upd2 -- python3 "$R/tools/time_update.py" --updates 10 > "$OUT/pmc_upd2.log" 2>&1
