#!/bin/bash
# round-3 experiment batch: wave timeline of the config-3 step, A/B of store policies and
# ablations (tools/stepbench), layout floors (tools/membench)
set -u
OUT=gpurun_out/r03c
mkdir -p $OUT
timeout -k 10 120 python3 tools/wave_trace.py --lib shippingenv_amd/_lib/trace/libshipenv_hip.so --config 3 > $OUT/wave_trace_c3.json || exit $?
timeout -k 10 120 python3 tools/wave_trace.py --lib shippingenv_amd/_lib/trace/libshipenv_hip.so --config 3 --steps 400 > $OUT/wave_trace_c3_400.json || exit $?
REGIMES="3:5:20 3:50:1000 4:50:1000" bash tools/ab_step.sh > $OUT/ab.jsonl 2> $OUT/ab.err || exit $?
timeout -k 10 120 tools/membench > $OUT/membench.txt 2>&1 || exit $?
