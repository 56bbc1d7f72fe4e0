#!/bin/bash
# rocprofv3 kernel trace of the driver's exact bench command, with the per-leg
# step-kernel averages (tools/kt_legs.py) beside the bench line printed under the
# profiler (run on the GPU box from the repo root):
#   bash tools/trace_driver.sh <tag> [extra bench.py args]
set -u
TAG=${1:-r03}
shift || true
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o kt_drv -- \
    python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 "$@" > "$OUT/kt_drv.log" 2>&1
rc=$?
cd "$R"
[ $rc -eq 0 ] || { tail -5 "$OUT/kt_drv.log"; exit $rc; }
grep '^{' "$OUT/kt_drv.log" > "$OUT/bench_under_rocprof.json"
python3 tools/kt_legs.py "$OUT/kt_drv_kernel_trace.csv" --bench "$OUT/bench_under_rocprof.json" > "$OUT/kt_legs.json"
rc=$?
rm -f "$OUT/kt_drv_kernel_trace.csv.gz"
gzip -f "$OUT/kt_drv_kernel_trace.csv"
exit $rc
