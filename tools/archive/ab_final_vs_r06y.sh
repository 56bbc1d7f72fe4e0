set -u
O=gpurun_out/r06ab; mkdir -p $O
for p in f32 bf16; do
  LIBS="shippingenv_amd/_lib/abl/y.so shippingenv_amd/_lib/abl/h.so" PREC=$p PREROLL=300 ROUNDS=4 timeout -k 10 600 bash tools/ab_policy.sh > $O/ab_$p.jsonl 2>$O/ab_$p.err || exit 1
  python3 tools/ab_summary.py $O/ab_$p.jsonl ms_per_launch
done
