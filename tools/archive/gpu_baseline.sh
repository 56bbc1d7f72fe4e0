set -u
mkdir -p gpurun_out
L=shippingenv_amd/_lib/libshipenv_hip.so
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
tail -2 gpurun_out/gpu_tests.log
for k in 1 2 3; do timeout -k 10 60 tools/stepbench --warm 5 --steps 20 $L || exit $?; done
for k in 1 2; do timeout -k 10 60 tools/stepbench --warm 50 --steps 1000 $L || exit $?; done
timeout -k 10 60 tools/stepbench --config 4 --warm 50 --steps 1000 $L || exit $?
timeout -k 10 60 tools/stepbench --config 4 --warm 5 --steps 20 $L || exit $?
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_drv.json 2> gpurun_out/bench_drv.err || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/bench_drv.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['config4']['roofline']['frac'])"
