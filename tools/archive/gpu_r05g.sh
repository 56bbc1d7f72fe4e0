# split-bf16 fp32 policy: timing, kernel trace and SQ counters (one pass each)
set -u
O=gpurun_out/${1:-r05g}; mkdir -p $O; R=$(pwd)
for r in 1 2; do
  timeout -k 10 120 python tools/time_policy.py --precision f32 --launches 20 >> $O/time_policy_f32.jsonl || exit 1
done
cat $O/time_policy_f32.jsonl
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O" -o kt_pol -- python3 "$R/tools/time_policy.py" --precision f32 --launches 10 > "$R/$O/kt_pol.log" 2>&1) || exit 1
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU \
   --output-format csv -d "$R/$O" -o pmc_pol32a -- python3 "$R/tools/time_policy.py" --precision f32 --launches 3 > "$R/$O/pmc_a.log" 2>&1) || exit 1
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE \
   --output-format csv -d "$R/$O" -o pmc_pol32b -- python3 "$R/tools/time_policy.py" --precision f32 --launches 3 > "$R/$O/pmc_b.log" 2>&1) || exit 1
ls $O
