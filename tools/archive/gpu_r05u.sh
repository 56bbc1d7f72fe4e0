#!/bin/bash
# round 5: is the back-to-back update loop host-bound? events vs host issue time (eager and
# graph) for the update builds, then the kernel trace of the product's eager loop
set -u
O=gpurun_out/${1:-r05u2}; mkdir -p $O
for lib in shippingenv_amd/_lib/ablu/u_bias.so shippingenv_amd/_lib/ablu/u_slot.so; do
  for g in "" "--graph"; do
    timeout -k 10 120 python tools/time_update.py --lib $lib $g >> $O/time_update.jsonl 2>>$O/err.log || exit 1
  done
done
R=$(pwd)
(export TMPDIR=/tmp && cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$R/$O/kt" -o upd --output-format csv -- python3 "$R/tools/time_update.py" --updates 100 > "$R/$O/kt.log" 2>&1) || exit 1
echo done
