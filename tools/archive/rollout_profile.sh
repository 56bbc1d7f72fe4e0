set -u
R=$(pwd); OUT=$R/gpurun_out/rollprof; mkdir -p $OUT; export TMPDIR=/tmp; cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o kt -- python3 $R/tools/time_rollout.py > $OUT/kt.log 2>&1 &&
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $OUT -o sq -- python3 $R/tools/time_rollout.py --launches 2 > $OUT/sq.log 2>&1
