set -u
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_policy.py tests/test_gpu_dqn.py > $O/tests.log 2>&1; echo "tests rc=$?"; tail -3 $O/tests.log
LIBS="shippingenv_amd/_lib/abl/fc3x0.so shippingenv_amd/_lib/abl/fc3x1.so" PREC=bf16 PREROLL=300 ROUNDS=4 timeout -k 10 400 bash tools/ab_policy.sh > $O/ab_fc3x.jsonl 2>$O/ab_fc3x.err; echo "ab rc=$?"; python3 tools/ab_summary.py $O/ab_fc3x.jsonl ms_per_launch
for lib in tb0 tb1; do timeout -k 10 120 python3 tools/time_policy.py --precision bf16 --launches 5 --preroll 300 --trace --lib shippingenv_amd/_lib/abl/$lib.so | cut -c 150- || exit 1; done
timeout -k 10 300 python3 tools/dqn_learning.py --n 4096 --iters 2000 --every 500 --updates-per-step 4 --preroll-train --torch --tag torch_u4p > $O/learn_torch_u4p.jsonl 2>/dev/null; echo "rc=$?"
timeout -k 10 300 python3 tools/dqn_learning.py --n 4096 --iters 2000 --every 500 --updates-per-step 4 --preroll-train --target-update-every 100 --tag u4p_t100 > $O/learn_u4p_t100.jsonl 2>/dev/null; echo "rc=$?"
for f in $O/learn_torch_u4p.jsonl $O/learn_u4p_t100.jsonl; do python3 -c "
import json,sys
for l in open('$f'):
    d=json.loads(l); print(d['tag'], d['eval'][:6], d['policy'][:6], d.get('iter'), d.get('epsilon'), round(d.get('loss') or 0,2), round(d['reward_per_env_step'],3), d['return_at_sea_start'] and round(d['return_at_sea_start'],1))
"; done
