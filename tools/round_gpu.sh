# One GPU call for a round's evidence (run on the GPU box from the repo root):
#   bash tools/round_gpu.sh <tag>
# GPU tests, smoke, the driver's bench command, the default bench, then the rocprofv3
# passes of tools/profile_round.sh. Each step has its own time limit; the chain stops
# at the first failure.
set -u
TAG=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" &&
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_drv.json 2> gpurun_out/bench_drv.err &&
timeout -k 10 300 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err &&
{ [ "${PROFILE:-1}" = "1" ] || exit 0; } &&
bash tools/profile_round.sh "$TAG"
