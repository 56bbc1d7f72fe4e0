set -u
O=gpurun_out/r06c; mkdir -p $O
timeout -k 10 300 python3 tools/dqn_learning.py --n 4096 --iters 2000 --every 500 --updates-per-step 4 --preroll-train --tag u4p > $O/learn_4096_u4p.jsonl 2>/dev/null; echo "rc=$?"
timeout -k 10 300 python3 tools/dqn_learning.py --n 4096 --iters 2000 --every 500 --updates-per-step 1 --preroll-train --tag u1p > $O/learn_4096_u1p.jsonl 2>/dev/null; echo "rc=$?"
timeout -k 10 300 python3 tools/dqn_learning.py --n 65536 --iters 2000 --every 500 --updates-per-step 1 --preroll-train --tag big > $O/learn_65536_u1p.jsonl 2>/dev/null; echo "rc=$?"
for f in $O/learn_4096_u4p.jsonl $O/learn_4096_u1p.jsonl $O/learn_65536_u1p.jsonl; do python3 -c "
import json,sys
for l in open('$f'):
    d=json.loads(l); print(d['tag'], d['eval'][:6], d['policy'][:6], d.get('iter'), d.get('epsilon'), round(d.get('loss') or 0,2), round(d['reward_per_env_step'],3), d['return_at_sea_start'] and round(d['return_at_sea_start'],1), round(d['share_at_sea_start'],2), d['episodes'])
"; done
for i in 1 2; do timeout -k 10 120 python3 tools/time_policy.py --precision bf16 --launches 5 --preroll 300 --trace --lib shippingenv_amd/_lib/abl/tb.so || exit 1; done
timeout -k 10 200 tools/stepbench --config 4 --steps 200 --preroll 1000 --floor 5 shippingenv_amd/_lib/libshipenv_hip.so || exit 1
timeout -k 10 200 tools/stepbench --config 3 --steps 200 --preroll 1000 --floor 3 shippingenv_amd/_lib/libshipenv_hip.so || exit 1
