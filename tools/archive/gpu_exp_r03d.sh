#!/bin/bash
set -u
OUT=gpurun_out/r03d
mkdir -p $OUT
REGIMES="3:5:20 3:50:1000 4:50:1000" bash tools/ab_step.sh > $OUT/ab.jsonl 2> $OUT/ab.err || exit $?
timeout -k 10 120 python3 tools/wave_trace.py --lib shippingenv_amd/_lib/trace1024/libshipenv_hip.so --config 3 > $OUT/wave_trace_c3_b1024.json || exit $?
timeout -k 10 120 tools/hbmcopy > $OUT/hbmcopy.jsonl || exit $?
