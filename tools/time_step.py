"""Time the step kernel of one library build (tuning / ablation helper).

    python tools/time_step.py [--lib path/to/libshipenv_hip.so] [--n N] [--config 3|4] [--steps K]

Prints one JSON line: wall us/step over K back-to-back launches, and the mean /
median of per-launch HIP-event durations on the launch stream.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--lib", default=None)
    p.add_argument("--n", type=int, default=1 << 20)
    p.add_argument("--config", type=int, default=3)
    p.add_argument("--steps", type=int, default=200)
    a = p.parse_args()
    from shippingenv_amd import _native

    if a.lib:
        _native.LIB_PATH = os.path.abspath(a.lib)
    from shippingenv_amd.maps import builtin_water
    from shippingenv_amd.vec import VecEnv, random_water_ports

    ports = random_water_ports(builtin_water(), 64, seed=3) if a.config == 4 else None
    env = VecEnv(a.n, seed=2026, ports=ports, auto_reset=a.config == 4, device="cuda:0")
    acts = torch.empty((a.steps, a.n), dtype=torch.int32, device="cuda:0")
    for t in range(a.steps):
        env.gen_actions(t, out=acts[t])
    env.reset()
    for t in range(20):
        env.step(acts[t])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(a.steps):
        env.step(acts[t])
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps * 1e6
    s = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(a.steps)]
    for t in range(a.steps):
        ev[t][0].record(s)
        env.step(acts[t])
        ev[t][1].record(s)
    torch.cuda.synchronize()
    us = np.array([x.elapsed_time(y) for x, y in ev]) * 1e3
    env.close()
    print(json.dumps({"lib": os.path.basename(a.lib or _native.LIB_PATH), "n": a.n,
                      "config": a.config, "wall_us": round(wall, 2),
                      "event_mean_us": round(float(us.mean()), 2),
                      "event_median_us": round(float(np.median(us)), 2),
                      "event_min_us": round(float(us.min()), 2)}), flush=True)


if __name__ == "__main__":
    main()
