#!/bin/bash
# round 4: GPU suite, done-list dense-layout A/B (config 4), T2 layout A/B (update)
set -u
OUT=gpurun_out/${1:-r04k}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $OUT/tests_gpu.log 2>&1 || exit $?
timeout -k 10 700 bash tools/ab_dense_r04.sh > $OUT/ab_dense.jsonl 2> $OUT/ab_dense.err || exit $?
timeout -k 10 600 bash tools/ab_upd_r04.sh $OUT/ab_upd || exit $?
