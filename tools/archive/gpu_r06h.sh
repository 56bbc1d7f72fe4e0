# round 6: fp32 policy sea-tile path A/B (visiting order on), then the policy tests
set -u
O=gpurun_out/r06h; mkdir -p $O
LIBS="shippingenv_amd/_lib/abl/xs0.so shippingenv_amd/_lib/abl/xs1.so" PREC=f32 PREROLL=300 ROUNDS=4 timeout -k 10 600 bash tools/ab_policy.sh > $O/ab_x3_sea.jsonl 2>$O/ab.err || exit 1
python3 tools/ab_summary.py $O/ab_x3_sea.jsonl ms_per_launch
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_policy.py > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; exit $rc
