"""Per-step kernel time over a long run (diagnostic): mean of HIP-event durations
in buckets of 50 steps, for config 3 or 4 at N envs.

    python tools/step_timeline.py --config 4 --steps 1000
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shippingenv_amd.maps import builtin_water  # noqa: E402
from shippingenv_amd.vec import VecEnv, random_water_ports  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", type=int, default=3)
    p.add_argument("--n", type=int, default=1 << 20)
    p.add_argument("--steps", type=int, default=1000)
    a = p.parse_args()
    ports = random_water_ports(builtin_water(), 64, seed=3) if a.config == 4 else None
    env = VecEnv(a.n, seed=2026, ports=ports, auto_reset=a.config == 4, device="cuda:0")
    acts = torch.empty((a.steps, a.n), dtype=torch.int32, device="cuda:0")
    for t in range(a.steps):
        env.gen_actions(t, out=acts[t])
    env.reset()
    s = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    done = torch.zeros(a.steps, dtype=torch.int64, device="cuda:0")
    cargo_pos = torch.zeros(a.steps, dtype=torch.int64, device="cuda:0")
    for t in range(a.steps):
        ev[t][0].record(s)
        env.step(acts[t])
        ev[t][1].record(s)
        done[t] = env.done.sum()
        cargo_pos[t] = (env.cargo > 0).sum()
    torch.cuda.synchronize()
    us = np.array([x.elapsed_time(y) for x, y in ev]) * 1e3
    d, c = done.cpu().numpy(), cargo_pos.cpu().numpy()
    out = []
    for b in range(0, a.steps, 50):
        out.append({"steps": f"{b}-{b + 49}", "us": round(float(us[b:b + 50].mean()), 2),
                    "done_per_step": int(d[b:b + 50].mean()), "cargo_gt0": int(c[b:b + 50].mean())})
    print(json.dumps({"config": a.config, "n": a.n, "buckets": out}))


if __name__ == "__main__":
    main()
