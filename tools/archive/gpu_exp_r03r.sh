#!/bin/bash
# N = 2^24: the Python forms (tools/diag/large_n_forms.py) and the C++ driver on one box
set -u
OUT=gpurun_out/r03r
mkdir -p $OUT
L=shippingenv_amd/_lib/libshipenv_hip.so
timeout -k 10 300 python3 tools/diag/large_n_forms.py > $OUT/large_n_forms.jsonl 2> $OUT/large_n_forms.err || exit $?
for warm in 5 1000; do
  timeout -k 10 120 tools/stepbench --config 3 --n 16777216 --warm $warm --steps 100 $L >> $OUT/stepbench.jsonl 2>> $OUT/stepbench.err || exit $?
done
