# round 6: the visiting order (policy_order_kernel): parity tests, then order off / on alternating
set -u
O=gpurun_out/r06g; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_policy.py tests/test_gpu_dqn.py > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for p in f32 bf16; do
    for o in 0 1; do
      SHIPENV_POLICY_ORDER=$o timeout -k 10 120 python3 tools/time_policy.py --precision $p --launches 20 --preroll 300 >> $O/ab_order.jsonl || exit 1
    done
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r06g/ab_order.jsonl"):
    r = json.loads(l); d[(r["precision"], r["order"])].append(r["ms_per_launch"])
for k, v in sorted(d.items()): print(k, sorted(v))
r = json.loads(open("gpurun_out/r06g/ab_order.jsonl").readline()); print("tiles with port:", r["wave32_with_port"], "ordered:", r["wave32_with_port_ordered"])
PY
for rep in 1 2 3; do
  for lib in sea0 sea1; do
    SHIPENV_POLICY_ORDER=1 timeout -k 10 120 python3 tools/time_policy.py --precision bf16 --launches 20 --preroll 300 --lib shippingenv_amd/_lib/abl/$lib.so >> $O/ab_sea.jsonl || exit 1
  done
done
python3 tools/ab_summary.py $O/ab_sea.jsonl ms_per_launch
for p in bf16 f32; do
  SHIPENV_POLICY_ORDER=1 timeout -k 10 120 python3 tools/time_policy.py --precision $p --launches 5 --preroll 300 --trace --lib shippingenv_amd/_lib/abl/tr.so >> $O/trace.jsonl || exit 1
done
cut -c 1-40,300-900 $O/trace.jsonl
