#!/bin/bash
# T1 / T2 phase stamps (SHIPENV_QTRACE builds) of the working tree's update, twice
set -u
OUT=${1:-gpurun_out/qtrace}
mkdir -p $OUT
for rep in 1 2; do
  timeout -k 10 120 python3 tools/qtrain_trace.py --lib shippingenv_amd/_lib/ab/lib_qt.so >> $OUT/qtrace.jsonl || exit $?
done
