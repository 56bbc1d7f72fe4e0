#!/bin/bash
# round 5: policy tests + bf16 / f32 policy A/B over shippingenv_amd/_lib/abl, then the
# config 3 / 5 / 6 / 4 split at 2^20 and 2^24 (tools/stepbench, the product library)
set -u
O=gpurun_out/${1:-r05r}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_policy.py tests/test_gpu_dqn.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
: > $O/ab.err
PREC=f32 ROUNDS=2 bash tools/ab_policy_r05.sh > $O/ab_policy_f32.jsonl 2>>$O/ab.err || exit 1
L=shippingenv_amd/_lib/libshipenv_hip.so
for rep in 1 2; do
  for c in 3 5 6 4; do
    timeout -k 10 60 tools/stepbench --config $c --preroll 1000 --warm 5 --steps 200 $L >> $O/c_split.jsonl || exit 1
    timeout -k 10 90 tools/stepbench --config $c --n 16777216 --preroll 1000 --warm 5 --steps 50 $L >> $O/c_split.jsonl || exit 1
  done
done
echo done
R=$(pwd)
(export TMPDIR=/tmp && cd /tmp &&
 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY \
   --output-format csv -d "$R/$O" -o pmc_sq_c4 -- python3 "$R/tools/prof_step.py" --config 4 --steps 20 > "$R/$O/pmc_sq_c4.log" 2>&1 &&
 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY \
   --output-format csv -d "$R/$O" -o pmc_sq_c3 -- python3 "$R/tools/prof_step.py" --config 3 --steps 20 > "$R/$O/pmc_sq_c3.log" 2>&1) || exit 1
echo pmc-done
