#!/bin/bash
# Collect the rocprofv3 evidence for one round (run on the GPU box from the repo root):
#   bash tools/profile_round.sh <tag>
# kernel-trace + stats per configuration, then PMC passes, one counter group per
# pass (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950). Each step has
# its own time limit and the chain stops at the first failure.
set -u
TAG=${1:-r01}
R=$(pwd)
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
PY="python3 $R/tools/prof_step.py"
run() {  # name, timeout, rocprofv3 args..., -- program
    local name=$1 t=$2
    shift 2
    echo "[profile] $name" >&2
    timeout -k 10 "$t" rocprofv3 "$@" > "$OUT/$name.log" 2>&1
}
cd /tmp
rocprofv3 -L > "$OUT/counters_available.txt" 2>&1 || true
run kt_bench 600 --kernel-trace --stats --output-format csv -d "$OUT" -o kt_bench -- python3 $R/bench.py --no-cpu &&
rm -f "$OUT/kt_bench_kernel_trace.csv" &&
grep '^{' "$OUT/kt_bench.log" > "$OUT/bench_under_rocprof.json" &&
run kt_c3 240 --kernel-trace --stats --output-format csv -d "$OUT" -o kt_c3 -- $PY --config 3 --steps 200 &&
run kt_c4 240 --kernel-trace --stats --output-format csv -d "$OUT" -o kt_c4 -- $PY --config 4 --steps 200 &&
run kt_big 240 --kernel-trace --stats --output-format csv -d "$OUT" -o kt_big -- $PY --config 3 --n 16777216 --steps 40 &&
run kt_roll 240 --kernel-trace --stats --output-format csv -d "$OUT" -o kt_roll -- python3 $R/tools/time_rollout.py --launches 10 &&
run kt_pol 240 --kernel-trace --stats --output-format csv -d "$OUT" -o kt_pol -- python3 $R/tools/time_policy.py --launches 20 &&
run kt_train 240 --kernel-trace --stats --output-format csv -d "$OUT" -o kt_train -- python3 $R/tools/time_train.py --iters 20 &&
run pmc_fetch_c4 240 --pmc FETCH_SIZE --output-format csv -d "$OUT" -o pmc_fetch_c4 -- $PY --config 4 --steps 20 &&
run pmc_write_c4 240 --pmc WRITE_SIZE --output-format csv -d "$OUT" -o pmc_write_c4 -- $PY --config 4 --steps 20 &&
run pmc_fetch_c3 240 --pmc FETCH_SIZE --output-format csv -d "$OUT" -o pmc_fetch_c3 -- $PY --config 3 --steps 20 &&
run pmc_write_c3 240 --pmc WRITE_SIZE --output-format csv -d "$OUT" -o pmc_write_c3 -- $PY --config 3 --steps 20 &&
run pmc_fetch_big 240 --pmc FETCH_SIZE --output-format csv -d "$OUT" -o pmc_fetch_big -- $PY --config 3 --n 16777216 --steps 10 &&
run pmc_write_big 240 --pmc WRITE_SIZE --output-format csv -d "$OUT" -o pmc_write_big -- $PY --config 3 --n 16777216 --steps 10 &&
run pmc_sq_c3 240 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT" -o pmc_sq_c3 -- $PY --config 3 --steps 20 &&
run pmc_sq2_c3 240 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY --output-format csv -d "$OUT" -o pmc_sq2_c3 -- $PY --config 3 --steps 20
rc=$?
echo "[profile] rc=$rc" >&2
exit $rc
