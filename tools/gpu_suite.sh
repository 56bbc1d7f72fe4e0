#!/bin/bash
# the GPU test suite, smoke() and the driver's bench command once, into gpurun_out/<tag>/
set -u
O=gpurun_out/${1:-suite}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/tests_gpu.log 2>&1 || { tail -40 $O/tests_gpu.log; exit 1; }
tail -2 $O/tests_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv.json 2> $O/bench_drv.err || { tail -20 $O/bench_drv.err; exit 1; }
echo suite-ok
