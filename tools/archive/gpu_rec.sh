set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dqn.py > gpurun_out/rec_tests.log 2>&1 || { tail -40 gpurun_out/rec_tests.log; exit 1; }
tail -3 gpurun_out/rec_tests.log
for r in 1 2; do
  timeout -k 10 120 python tools/time_train.py --pair >> gpurun_out/rec_time.jsonl
  timeout -k 10 120 python tools/time_train.py >> gpurun_out/rec_time.jsonl
done
cat gpurun_out/rec_time.jsonl
