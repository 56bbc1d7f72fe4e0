#!/bin/bash
# the round's evidence on the final code: the GPU suite, smoke(), the driver's bench command twice,
# its rocprofv3 kernel trace (tools/trace_driver.sh -> kt_legs.json) and the PMC traffic passes
# (tools/pmc_traffic.sh), the size sweep and the update / policy SQ counters, all from one box
set -u
TAG=${1:-r06z}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $OUT/tests_gpu.log 2>&1 || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_drv.json 2> $OUT/bench_drv.err || exit $?
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_drv2.json 2> $OUT/bench_drv2.err || exit $?
bash tools/trace_driver.sh $TAG || exit $?
bash tools/pmc_traffic.sh $TAG || exit $?
# throughput against N (config 3: 2^14..2^25, config 4: 2^18..2^24), then the SQ counters of the
# DQN update's kernels and of the bf16 policy kernel (one pass each)
timeout -k 10 400 python3 tools/size_sweep.py --out $OUT/size_sweep.json > $OUT/size_sweep.log 2>&1 || exit $?
bash tools/pmc_update.sh $TAG || exit $?
R=$(pwd)
(export TMPDIR=/tmp && cd /tmp &&
 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU \
   --output-format csv -d "$R/$OUT" -o pmc_pol -- python3 "$R/tools/time_policy.py" --preroll 300 --launches 3 > "$R/$OUT/pmc_pol.log" 2>&1) || exit $?
(export TMPDIR=/tmp && cd /tmp &&
 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU \
   --output-format csv -d "$R/$OUT" -o pmc_pol32a -- python3 "$R/tools/time_policy.py" --precision f32 --preroll 300 --launches 3 > "$R/$OUT/pmc_pol32a.log" 2>&1 &&
 timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
   --output-format csv -d "$R/$OUT" -o pmc_pol32b -- python3 "$R/tools/time_policy.py" --precision f32 --preroll 300 --launches 3 > "$R/$OUT/pmc_pol32b.log" 2>&1) || exit $?
# round 6: the bf16 policy's wait counters, the rollout kernel's SQ counters, config 3 / 4 against
# bare streaming kernels of their bytes (stepbench --floor), the N = 1 stepper wave
bash tools/pmc_policy_bf16.sh $TAG || exit $?
bash tools/pmc_rollout.sh $TAG || exit $?
timeout -k 10 200 tools/stepbench --config 4 --steps 200 --preroll 1000 --floor 5 shippingenv_amd/_lib/libshipenv_hip.so > $OUT/c4_floor.txt 2>&1 || exit $?
timeout -k 10 200 tools/stepbench --config 3 --steps 200 --preroll 1000 --floor 5 shippingenv_amd/_lib/libshipenv_hip.so > $OUT/c3_floor.txt 2>&1 || exit $?
timeout -k 10 120 python3 tools/time_server.py > $OUT/time_server.jsonl 2>&1 || exit $?
echo final-ok
