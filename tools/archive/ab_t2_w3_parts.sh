#!/bin/bash
# T2's W3 rows in 2 workgroups (a, the code before) or 4 (q4): back-to-back updates alternating,
# then the update's GPU tests on the product build (q4)
set -u
OUT=gpurun_out/${1:-r06w3}
mkdir -p $OUT
L=shippingenv_amd/_lib/ab
for rep in 1 2 3 4; do
  for v in a q4; do
    timeout -k 10 120 python3 tools/time_update.py --lib $L/lib_$v.so | sed "s/^{/{\"v\": \"$v\", /" >> $OUT/ab.jsonl || exit $?
  done
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dqn.py > $OUT/tests_dqn.log 2>&1 || exit $?
echo ab-ok
