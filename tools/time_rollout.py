"""bench.py's rollouts leg alone (se_rollout: 2^20 MCTS random rollouts of up to 100 counted
steps from config-3 states after 50 steps), for kernel traces and PMC passes
(tools/pmc_rollout.sh). One JSON line: launches, counted steps, events ms per launch.

    python tools/time_rollout.py [--n 1048576] [--launches 3]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=1 << 20)
    p.add_argument("--launches", type=int, default=3)
    p.add_argument("--seed", type=int, default=2026)
    a = p.parse_args()
    from shippingenv_amd.vec import VecEnv

    env = VecEnv(a.n, seed=a.seed, device="cuda:0")
    env.reset()
    for t in range(50):
        env.step(env.gen_actions(t))
    src = torch.arange(a.n, dtype=torch.int32, device=env.device)
    env.rollout(src, max_steps=100, rollout_base=0)  # warm
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    kept = []
    e0.record()
    for k in range(a.launches):
        kept.append(env.rollout(src, max_steps=100, rollout_base=(2 + k) * a.n)[1])
    e1.record()
    torch.cuda.synchronize()
    total = int(sum(int(s.sum().item()) for s in kept))
    print(json.dumps({"n": a.n, "launches": a.launches, "counted_steps": total,
                      "steps_per_launch": total / a.launches,
                      "kernel_ms": round(e0.elapsed_time(e1) / a.launches, 4)}), flush=True)
    env.close()


if __name__ == "__main__":
    main()
