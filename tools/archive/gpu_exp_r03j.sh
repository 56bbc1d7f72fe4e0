#!/bin/bash
set -u
OUT=gpurun_out/r03j
mkdir -p $OUT
for rep in 1 2; do
  for lib in shippingenv_amd/_lib/abl/a_base.so shippingenv_amd/_lib/abl/b_st1.so; do
    timeout -k 10 120 python3 tools/diag/map_size_effect.py --lib $lib >> $OUT/map_size.jsonl || exit $?
  done
done
bash tools/ab_step_n.sh > $OUT/ab.jsonl 2> $OUT/ab.err || exit $?
