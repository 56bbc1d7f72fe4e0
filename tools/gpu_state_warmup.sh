#!/bin/bash
# The short-run diagnosis (tools/diag/state_vs_warmup.py): each case in a fresh process.
#   bash tools/gpu_state_warmup.sh <outdir>
set -u
OUT=${1:-gpurun_out/state_warmup}
mkdir -p "$OUT"
D=tools/diag/state_vs_warmup.py
S=/tmp/shipenv_s1000.pt
timeout -k 10 120 python3 $D --save $S > "$OUT/save.json" &&
for c in reset_cold steady_cold reset_warm steady_warm reset_cold steady_cold; do
    L=""
    case $c in steady_*) L="--load $S";; esac
    timeout -k 10 120 python3 $D --case $c $L >> "$OUT/cases.jsonl" || exit $?
done
