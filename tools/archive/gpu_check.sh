# One GPU call: the GPU test suite, then (unless a test crashed, timed out or the
# run faulted) the step A/B of tools/ab_step.sh. Test failures (rc 1) still let
# the timing run; anything else stops the call.
set -u
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-400} python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  ${TESTS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -25 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
[ "${AB:-1}" = "1" ] && { bash tools/ab_step.sh || exit $?; }
exit $rc
