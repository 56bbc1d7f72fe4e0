#!/bin/bash
# round 4: the step at 2^21 envs (config 3 and 4), the default grid (one group per thread, 2048
# workgroups: two dispatch rounds) against a 1024-workgroup grid of two groups per thread,
# alternating, three rounds (tools/size_sweep.py)
set -u
OUT=${1:-gpurun_out/ab_2p21}
mkdir -p $OUT
for rep in 1 2 3; do
  for b in default 1024; do
    if [ $b = default ]; then
      timeout -k 10 120 python3 tools/size_sweep.py --log2n 21 --log2n4 21 --out $OUT/sweep_${b}_$rep.json > /dev/null || exit $?
    else
      SHIPENV_STEP_BLOCKS=$b timeout -k 10 120 python3 tools/size_sweep.py --log2n 21 --log2n4 21 --out $OUT/sweep_${b}_$rep.json > /dev/null || exit $?
    fi
  done
done
