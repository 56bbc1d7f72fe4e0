# round 6: fp32 policy sea tiles with fc3 rows 0-3 as three stacked chains (SHIPENV_X3_STACK) A/B
set -u
O=gpurun_out/r06p; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_policy.py tests/test_gpu_dqn.py > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="shippingenv_amd/_lib/abl/st0.so shippingenv_amd/_lib/abl/st1.so" PREC=f32 PREROLL=300 ROUNDS=4 timeout -k 10 600 bash tools/ab_policy.sh > $O/ab_f32.jsonl 2>$O/ab_f32.err || exit 1
python3 tools/ab_summary.py $O/ab_f32.jsonl ms_per_launch
