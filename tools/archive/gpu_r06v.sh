# round 6: the bf16 policy's order list in LDS (l) vs in global scratch (g)
set -u
O=gpurun_out/r06v; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_policy.py tests/test_gpu_dqn.py > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="shippingenv_amd/_lib/abl/g.so shippingenv_amd/_lib/abl/l.so" PREC=bf16 PREROLL=300 ROUNDS=5 timeout -k 10 600 bash tools/ab_policy.sh > $O/ab_bf16.jsonl 2>$O/ab_bf16.err || exit 1
python3 tools/ab_summary.py $O/ab_bf16.jsonl ms_per_launch
timeout -k 10 120 python3 tools/time_policy.py --precision bf16 --launches 5 --preroll 300 --trace --lib shippingenv_amd/_lib/abl/tr.so >> $O/trace.jsonl || exit 1
python3 -c "
import json
for l in open('$O/trace.jsonl'):
    d=json.loads(l); print(d['precision'], d['ms_per_launch'], 'image', d['us_image_median'], 'wave', d['us_wave_median'], 'end', d['us_end_max'])"
