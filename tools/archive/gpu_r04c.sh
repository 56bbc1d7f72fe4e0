#!/bin/bash
# round 4: wall-time forms (native vs per-call issue, host wait settings), config-4 cost split at
# 2^24, policy / update A/B
set -u
OUT=gpurun_out/${1:-r04c}
mkdir -p $OUT
timeout -k 10 400 python3 tools/diag/wall_forms.py --reps 12 --settings default,active_wait > $OUT/wall_forms.jsonl 2> $OUT/wall_forms.err || exit $?
timeout -k 10 400 bash tools/ab_c4split_r04.sh > $OUT/c4split.jsonl 2> $OUT/c4split.err || exit $?
timeout -k 10 700 bash tools/ab_pol_upd_r04.sh $OUT/ab_pol_upd || exit $?
