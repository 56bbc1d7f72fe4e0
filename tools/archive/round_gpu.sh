# One GPU call for a round's evidence (run on the GPU box from the repo root):
#   bash tools/round_gpu.sh <tag>
# GPU tests, smoke, the driver's bench command, its rocprofv3 kernel trace with the
# per-leg averages (tools/trace_driver.sh), the default bench, then the rocprofv3 passes of
# tools/profile_round.sh. Each step has its own time limit; the chain stops at the first
# failure.
set -u
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1
rc=$?
tail -3 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_drv.json 2> $OUT/bench_drv.err &&
bash tools/trace_driver.sh $TAG &&
timeout -k 10 400 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err &&
{ [ "${PROFILE:-1}" = "1" ] || exit 0; } &&
bash tools/profile_round.sh "$TAG"
