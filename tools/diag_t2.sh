#!/bin/bash
# T2 (qtrain_adam_kernel) diagnostics: phase stamps per block kind (SHIPENV_QTRACE build at
# shippingenv_amd/_lib/ab/lib_qt.so), back-to-back update time, and T2's HBM traffic
# (FETCH_SIZE / WRITE_SIZE, one counter per pass) and TCC hit counts over 10 updates
set -u
TAG=${1:-r06t2}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
  timeout -k 10 120 python3 tools/qtrain_trace.py --lib shippingenv_amd/_lib/ab/lib_qt.so >> $OUT/qtrace.jsonl || exit $?
done
timeout -k 10 120 python3 tools/time_update.py >> $OUT/time_update.jsonl || exit $?
export TMPDIR=/tmp
cd /tmp
for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum"; do
  n=$(echo $c | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT" -o pmc_$n -- python3 "$R/tools/time_update.py" --updates 10 > "$OUT/pmc_$n.log" 2>&1 || exit $?
done
echo t2-ok
