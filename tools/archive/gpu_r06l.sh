# round 6: the resident stepper wave with the world in LDS: timing, compat tests, config 1
set -u
O=gpurun_out/r06l; mkdir -p $O
timeout -k 10 120 python3 tools/time_server.py > $O/time_server.jsonl 2>&1; rc=$?; cat $O/time_server.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_compat_gpu.py -s > $O/compat.log 2>&1; rc=$?; grep -E "compat step|passed|failed|Error" $O/compat.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv.json 2> $O/bench_drv.err || { tail -20 $O/bench_drv.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_drv.json').read().strip().splitlines()[-1]); print(json.dumps(d['config1']))"
