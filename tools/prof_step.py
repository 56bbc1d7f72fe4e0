"""Minimal driver for rocprofv3 runs: steps one configuration K times.

    rocprofv3 --kernel-trace --stats -- python tools/prof_step.py --config 3 --steps 100
    rocprofv3 --pmc FETCH_SIZE -- python tools/prof_step.py --config 3 --steps 20
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from shippingenv_amd.maps import builtin_water  # noqa: E402
from shippingenv_amd.vec import VecEnv, random_water_ports  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", type=int, default=3, choices=(3, 4))
    p.add_argument("--n", type=int, default=1 << 20)
    p.add_argument("--steps", type=int, default=100)
    a = p.parse_args()
    ports = random_water_ports(builtin_water(), 64, seed=3) if a.config == 4 else None
    env = VecEnv(a.n, seed=2026, ports=ports, auto_reset=a.config == 4, device="cuda:0")
    acts = torch.empty((a.steps, a.n), dtype=torch.int32, device="cuda:0")
    for t in range(a.steps):
        env.gen_actions(t, out=acts[t])
    env.reset()
    torch.cuda.synchronize()
    for t in range(a.steps):
        env.step(acts[t])
    torch.cuda.synchronize()
    env.close()
    print(f"done config={a.config} n={a.n} steps={a.steps}")


if __name__ == "__main__":
    main()
