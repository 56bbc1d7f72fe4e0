#!/bin/bash
# PMC traffic passes (one counter per pass; FETCH_SIZE and WRITE_SIZE apart, MI355X_MICROARCH
# §HBM) for config 3 and config 4 at 2^20 and 2^24 (tools/prof_step.py), then the SQ counters of
# config 3, into gpurun_out/prof_<tag>/ (tools/summarize_profiles.py condenses it)
set -u
TAG=${1:-r04}
R=$(pwd)
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
PY="python3 $R/tools/prof_step.py"
run() {
    local name=$1
    shift
    echo "[pmc] $name" >&2
    timeout -s KILL 120 rocprofv3 "$@" > "$OUT/$name.log" 2>&1
}
cd /tmp
run pmc_fetch_c3 --pmc FETCH_SIZE --output-format csv -d "$OUT" -o pmc_fetch_c3 -- $PY --config 3 --steps 20 &&
run pmc_write_c3 --pmc WRITE_SIZE --output-format csv -d "$OUT" -o pmc_write_c3 -- $PY --config 3 --steps 20 &&
run pmc_fetch_c4 --pmc FETCH_SIZE --output-format csv -d "$OUT" -o pmc_fetch_c4 -- $PY --config 4 --steps 20 &&
run pmc_write_c4 --pmc WRITE_SIZE --output-format csv -d "$OUT" -o pmc_write_c4 -- $PY --config 4 --steps 20 &&
run pmc_fetch_big --pmc FETCH_SIZE --output-format csv -d "$OUT" -o pmc_fetch_big -- $PY --config 3 --n 16777216 --steps 10 &&
run pmc_write_big --pmc WRITE_SIZE --output-format csv -d "$OUT" -o pmc_write_big -- $PY --config 3 --n 16777216 --steps 10 &&
run pmc_fetch_c4big --pmc FETCH_SIZE --output-format csv -d "$OUT" -o pmc_fetch_c4big -- $PY --config 4 --n 16777216 --steps 10 &&
run pmc_write_c4big --pmc WRITE_SIZE --output-format csv -d "$OUT" -o pmc_write_c4big -- $PY --config 4 --n 16777216 --steps 10 &&
run pmc_sq_c3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT" -o pmc_sq_c3 -- $PY --config 3 --steps 20 &&
run pmc_sq2_c3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY --output-format csv -d "$OUT" -o pmc_sq2_c3 -- $PY --config 3 --steps 20
rc=$?
cd "$R"
echo "[pmc] rc=$rc" >&2
exit $rc
