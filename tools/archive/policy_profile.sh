#!/bin/bash
# rocprofv3 kernel trace + SQ counters of the fused policy step (GPU box).
set -u
R=$(pwd); OUT=$R/gpurun_out/polprof; mkdir -p $OUT; export TMPDIR=/tmp; cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o kt -- python3 $R/tools/time_policy.py > $OUT/kt.log 2>&1 &&
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $OUT -o sq1 -- python3 $R/tools/time_policy.py --launches 3 > $OUT/sq1.log 2>&1 &&
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $OUT -o sq2 -- python3 $R/tools/time_policy.py --launches 3 > $OUT/sq2.log 2>&1
