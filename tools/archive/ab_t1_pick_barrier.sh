#!/bin/bash
# T1: the other waves' weight loads behind a barrier after wave 0 issues its minibatch picks (b), or
# fc2's operand loads moved after the input barrier (c), against the code before (a) (VARS): input sub-phase stamps (SHIPENV_QTRACE=2 builds), back-to-back
# updates alternating, then the update's GPU tests on the product build (b)
set -u
OUT=gpurun_out/${1:-r06pb}
mkdir -p $OUT
L=shippingenv_amd/_lib/ab
for v in ${VARS:-a b}; do
  timeout -k 10 120 python3 tools/qtrain_trace.py --inputs --lib $L/lib_qt_$v.so | sed "s/^{/{\"v\": \"$v\", /" >> $OUT/qtrace.jsonl || exit $?
done
for rep in 1 2 3; do
  for v in ${VARS:-a b}; do
    timeout -k 10 120 python3 tools/time_update.py --lib $L/lib_$v.so | sed "s/^{/{\"v\": \"$v\", /" >> $OUT/ab.jsonl || exit $?
  done
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dqn.py > $OUT/tests_dqn.log 2>&1 || exit $?
echo ab-ok
