#!/bin/bash
# The short-run diagnosis (tools/diag/state_vs_warmup.py): each case in a fresh process,
# twice, in alternating order; then the reset case with a longer active-wait spin.
#   bash tools/gpu_state_warmup.sh <outdir>
set -u
OUT=${1:-gpurun_out/state_warmup}
mkdir -p "$OUT"
D=tools/diag/state_vs_warmup.py
S=/tmp/shipenv_s1000.pt
timeout -k 10 120 python3 $D --save $S > "$OUT/save.json" || exit $?
for rep in 1 2; do
  for c in reset_cold steady_cold reset_warm steady_warm; do
    L=""
    case $c in steady_*) L="--load $S";; esac
    timeout -k 10 120 python3 $D --case $c $L >> "$OUT/cases.jsonl" || exit $?
  done
done
for rep in 1 2; do
  ROC_ACTIVE_WAIT_TIMEOUT=100000 timeout -k 10 120 python3 $D --case reset_cold >> "$OUT/cases.jsonl" || exit $?
  timeout -k 10 120 python3 $D --case reset_cold >> "$OUT/cases.jsonl" || exit $?
done
