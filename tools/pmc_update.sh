#!/bin/bash
# SQ counters of the DQN update's kernels (tools/diag/update_forms.py, eager), one pass
set -u
R=$(pwd)
OUT=$R/gpurun_out/${1:-r03x}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES \
    --output-format csv -d "$OUT" -o pmc_upd -- python3 "$R/tools/diag/update_forms.py" --forms eager --iters 10 > "$OUT/pmc_upd.log" 2>&1
