# round 6: the order's loads issued before the image is staged (o2) vs the dependent chain (o1)
set -u
O=gpurun_out/r06r; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_policy.py tests/test_gpu_dqn.py > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for p in f32 bf16; do
  LIBS="shippingenv_amd/_lib/abl/o1.so shippingenv_amd/_lib/abl/o2.so" PREC=$p PREROLL=300 ROUNDS=4 timeout -k 10 600 bash tools/ab_policy.sh > $O/ab_$p.jsonl 2>$O/ab_$p.err || exit 1
  python3 tools/ab_summary.py $O/ab_$p.jsonl ms_per_launch
done
for p in bf16 f32; do timeout -k 10 120 python3 tools/time_policy.py --precision $p --launches 5 --preroll 300 --trace --lib shippingenv_amd/_lib/abl/tr.so >> $O/trace.jsonl || exit 1; done
python3 -c "
import json
for l in open('$O/trace.jsonl'):
    d=json.loads(l); print(d['precision'], d['ms_per_launch'], 'image', d['us_image_median'], 'wave', d['us_wave_median'], 'end', d['us_end_max'])"
