#!/bin/bash
# round 4: the GPU suite on the working tree, then the slab A/B
set -u
OUT=gpurun_out/${1:-r04d}
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $OUT/tests_gpu.log 2>&1 || exit $?
timeout -k 10 600 bash tools/ab_slab_r04.sh > $OUT/ab_slab.jsonl 2> $OUT/ab_slab.err || exit $?
timeout -k 10 500 bash tools/ab_upd_r04.sh $OUT/ab_upd || exit $?
