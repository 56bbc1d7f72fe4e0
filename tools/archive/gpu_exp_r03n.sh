#!/bin/bash
# issue forms alternated in one process, plain and under the kernel tracer
set -u
R=$(pwd)
OUT=$R/gpurun_out/r03n
mkdir -p $OUT
timeout -k 10 200 python3 tools/diag/issue_forms.py > $OUT/issue_forms.jsonl 2> $OUT/issue_forms.err || exit $?
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o kt_forms -- \
    python3 "$R/tools/diag/issue_forms.py" > "$OUT/issue_forms_prof.jsonl" 2> $OUT/issue_forms_prof.err || exit $?
gzip -f "$OUT/kt_forms_kernel_trace.csv"
