#!/bin/bash
# the 16 x 16 policy kernels (SHIPENV_POLICY16, pipelined and not) against the 32 x 32 one:
# the builds timed alternately (tools/time_policy.py), then the policy and DQN GPU tests on
# the 16 x 16 builds. A test failure is recorded and the script goes on; a fault, abort or
# time limit ends it.
set -u
OUT=gpurun_out/${1:-r04c}
mkdir -p $OUT
D=shippingenv_amd/_lib/abl
fatal() { case $1 in 124|134|137|139) exit $1;; esac; }
for rep in 1 2 3; do for lib in $D/p32.so $D/p16.so $D/p16np.so; do
  timeout -k 10 120 python3 tools/time_policy.py --lib $lib --launches 50 >> $OUT/policy_ab.jsonl || exit $?
done; done
SHIPENV_LIB=$D/p16.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_policy.py tests/test_gpu_dqn.py -m gpu > $OUT/tests_p16.log 2>&1; rc=$?; echo "p16 tests rc=$rc"; fatal $rc
SHIPENV_LIB=$D/p16np.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_policy.py -m gpu > $OUT/tests_p16np.log 2>&1; rc=$?; echo "p16np tests rc=$rc"; fatal $rc
exit 0
