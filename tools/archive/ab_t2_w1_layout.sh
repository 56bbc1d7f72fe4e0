#!/bin/bash
# T2's W1 blocks: dW1 / db1 partials [tiles][128][6] + [tiles][128] (a) against [128][tiles][8] (b):
# phase stamps of both (SHIPENV_QTRACE builds), back-to-back updates alternating, then the
# update's GPU tests on the product build (VARS="a b c": c = b with XCD-aware tile positions)
set -u
OUT=gpurun_out/${1:-r06t2b}
mkdir -p $OUT
L=shippingenv_amd/_lib/ab
for v in ${VARS:-a b}; do
  QT_W3_BLOCKS_PER_ROW=$([ $v = e -o $v = f ] && echo 2 || echo 1) timeout -k 10 120 python3 tools/qtrain_trace.py --lib $L/lib_qt_$v.so | sed "s/^{/{\"v\": \"$v\", /" >> $OUT/qtrace.jsonl || exit $?
done
for rep in 1 2 3; do
  for v in ${VARS:-a b}; do
    timeout -k 10 120 python3 tools/time_update.py --lib $L/lib_$v.so | sed "s/^{/{\"v\": \"$v\", /" >> $OUT/ab.jsonl || exit $?
  done
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dqn.py > $OUT/tests_dqn.log 2>&1 || exit $?
echo ab-ok
# PMC=1: T2's L2 requests and fabric reads per variant (one pass each)
if [ "${PMC:-0}" = 1 ]; then
  R=$(pwd)
  for v in ${VARS:-a b}; do
    (export TMPDIR=/tmp && cd /tmp && timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum --output-format csv \
       -d "$R/$OUT" -o pmc_$v -- python3 "$R/tools/time_update.py" --updates 10 --lib "$R/$L/lib_$v.so" > "$R/$OUT/pmc_$v.log" 2>&1) || exit $?
  done
  echo pmc-ok
fi
