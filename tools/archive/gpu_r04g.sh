#!/bin/bash
# round 4: done-list padding A/B (config 4), the GPU suite, T1 partial-store A/B (update)
set -u
OUT=gpurun_out/${1:-r04g}
mkdir -p $OUT
timeout -k 10 700 bash tools/ab_donepad_r04.sh > $OUT/ab_donepad.jsonl 2> $OUT/ab_donepad.err || exit $?
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $OUT/tests_gpu.log 2>&1 || exit $?
timeout -k 10 600 bash tools/ab_upd_r04.sh $OUT/ab_upd || exit $?
