"""Time se_rollout (MCTS random rollouts) on one GPU: m rollouts x max_steps.

    python tools/time_rollout.py [--m M] [--steps S] [--launches K]
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
    p.add_argument("--m", type=int, default=1 << 20)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--launches", type=int, default=5)
    a = p.parse_args()
    from shippingenv_amd.vec import VecEnv

    env = VecEnv(a.m, seed=2026, device="cuda:0")
    env.reset()
    for t in range(50):
        env.step(env.gen_actions(t))
    src = torch.arange(a.m, dtype=torch.int32, device="cuda:0")
    env.rollout(src, max_steps=a.steps)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    tot = 0
    for k in range(a.launches):
        _, steps, status = env.rollout(src, max_steps=a.steps, rollout_base=(k + 1) * a.m)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.launches
    print(json.dumps({"m": a.m, "max_steps": a.steps, "ms_per_launch": round(ms, 4),
                      "mean_steps": float(steps.float().mean()),
                      "status_counts": torch.bincount(status.long(), minlength=5).tolist()}))


if __name__ == "__main__":
    main()
