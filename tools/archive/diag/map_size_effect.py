"""How much the world image's staging costs the config-3 step at N = 2^20 (diagnostic):
the same step on the 100 x 100 reference map and on small all-water maps whose image fits
one staging row, with the library at --lib (a build with -DSHIPENV_STAGE_MIN_WORDS=1024
stages one 4 KB row per workgroup instead of three).

    python tools/diag/map_size_effect.py --lib shippingenv_amd/_lib/abl/x.so

One JSON line per map: us per step over K back-to-back launches (HIP events), steps 50..1050.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--lib")
    p.add_argument("--n", type=int, default=1 << 20)
    p.add_argument("--steps", type=int, default=300)
    a = p.parse_args()
    from shippingenv_amd import _native

    if a.lib:
        _native.LIB_PATH = os.path.abspath(a.lib)
    from shippingenv_amd.vec import VecEnv

    maps = {"ref100": (None, None)}
    for side in (48, 32):
        water = np.ones((side, side), np.uint8)
        water[side // 2, :side // 3] = 0  # a little ground
        ports = [[3, 3], [side - 4, 5], [side // 2 + 3, side - 6], [5, side - 5], [side - 6, side - 6]]
        maps[f"water{side}"] = (water, ports)
    for name, (water, ports) in maps.items():
        env = VecEnv(a.n, seed=2026, water=water, ports=ports, device="cuda:0")
        acts = torch.empty((64, a.n), dtype=torch.int32, device="cuda:0")
        for t in range(64):
            env.gen_actions(t, out=acts[t])
        env.reset()
        for t in range(50):
            env.step(acts[t % 64])
        torch.cuda.synchronize()
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for t in range(a.steps):
            env.step(acts[t % 64])
        e1.record(s)
        torch.cuda.synchronize()
        print(json.dumps({"lib": os.path.basename(a.lib or "default"), "map": name,
                          "us_per_step": round(e0.elapsed_time(e1) * 1e3 / a.steps, 3)}))
        env.close()


if __name__ == "__main__":
    main()
