#!/bin/bash
# round 4: the headline's wall time beyond its kernels
set -u
OUT=gpurun_out/${1:-r04w}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 tools/diag/wall_forms.py --reps 15 > $OUT/wall_forms.jsonl 2> $OUT/wall_forms.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $OUT/rt -o run -- \
    python3 tools/diag/wall_forms.py --child --reps 4 > $OUT/rt_child.json 2> $OUT/rt_child.err || exit $?
