#!/bin/bash
# SQ counters of rollout_kernel (tools/time_rollout.py: 2^20 rollouts x 3 launches + 1 warm):
# instruction counts, wave cycles and the wait / issue split, one pass per counter group
set -u
OUT=gpurun_out/${1:-pmc_rollout}
mkdir -p $OUT
R=$(pwd)
(export TMPDIR=/tmp && cd /tmp &&
 timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT" -o kt_roll -- python3 "$R/tools/time_rollout.py" > "$R/$OUT/kt_roll.log" 2>&1 &&
 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
   --output-format csv -d "$R/$OUT" -o pmc_roll_a -- python3 "$R/tools/time_rollout.py" > "$R/$OUT/pmc_roll_a.log" 2>&1 &&
 timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE \
   --output-format csv -d "$R/$OUT" -o pmc_roll_b -- python3 "$R/tools/time_rollout.py" > "$R/$OUT/pmc_roll_b.log" 2>&1) || exit $?
echo pmc-rollout-ok
