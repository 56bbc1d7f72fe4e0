#!/bin/bash
# Time the policy kernel of every library under shippingenv_amd/_lib/abl (two rounds).
set -u
mkdir -p gpurun_out
for rep in 1 2; do for lib in shippingenv_amd/_lib/abl/*.so; do
  timeout -k 10 120 python3 tools/time_policy.py --lib $lib --launches 50 >> gpurun_out/polab.jsonl || exit $?
done; done
