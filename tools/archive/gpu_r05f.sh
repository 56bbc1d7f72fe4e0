set -u
O=gpurun_out/${1:-r05f}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_policy.py > $O/tests_policy.log 2>&1; rc=$?
tail -30 $O/tests_policy.log
for r in 1 2; do
  for m in split mfma; do
    SHIPENV_POLICY_F32=$m timeout -k 10 120 python tools/time_policy.py --precision f32 --launches 20 >> $O/time_policy_f32.jsonl || exit 1
  done
done
cat $O/time_policy_f32.jsonl
exit $rc
