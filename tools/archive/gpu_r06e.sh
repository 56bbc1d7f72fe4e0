# round 6: where the policy launches' tail is (per XCD / per SIMD end times), bf16 and fp32
set -u
O=gpurun_out/r06e; mkdir -p $O
for p in bf16 f32; do
  timeout -k 10 120 python3 tools/time_policy.py --precision $p --launches 5 --preroll 300 --trace --lib shippingenv_amd/_lib/abl/tr.so >> $O/tail.jsonl || exit 1
done
cut -c 150- $O/tail.jsonl
