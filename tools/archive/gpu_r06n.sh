# round 6: the visiting order built inside the policy kernels (order_chunk) vs its own kernel
set -u
O=gpurun_out/r06n; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_policy.py tests/test_gpu_dqn.py > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for p in f32 bf16; do
  LIBS="shippingenv_amd/_lib/abl/sep.so shippingenv_amd/_lib/abl/fused.so" PREC=$p PREROLL=300 ROUNDS=4 timeout -k 10 600 bash tools/ab_policy.sh > $O/ab_$p.jsonl 2>$O/ab_$p.err || exit 1
  python3 tools/ab_summary.py $O/ab_$p.jsonl ms_per_launch
done
