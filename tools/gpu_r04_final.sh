#!/bin/bash
# round-4 evidence on the final code: the GPU suite, smoke(), the driver's bench command twice,
# its rocprofv3 kernel trace (tools/trace_driver.sh -> kt_legs.json) and the PMC traffic passes
# (tools/pmc_r04.sh), all from one box
set -u
TAG=${1:-r04z}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $OUT/tests_gpu.log 2>&1 || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_drv.json 2> $OUT/bench_drv.err || exit $?
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_drv2.json 2> $OUT/bench_drv2.err || exit $?
bash tools/trace_driver.sh $TAG || exit $?
bash tools/pmc_r04.sh $TAG || exit $?
