"""The config-3 step at N = 2^24 from Python, in the forms bench.py's large_n legs could
take (diagnostic): from reset and after a 1000-step pre-roll, on torch's current stream and
on a stream of its own; 100 timed launches after 5 warm-up, HIP events around them.

    python tools/diag/large_n_forms.py [--n 16777216]
One JSON line per form: us per step.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def run(n, preroll, side, steps=100, warm=5):
    from shippingenv_amd.vec import VecEnv

    s = torch.cuda.Stream() if side else torch.cuda.current_stream()
    with torch.cuda.stream(s):
        env = VecEnv(n, seed=2026, device="cuda:0")
        acts = torch.empty((warm + steps, n), dtype=torch.int32, device="cuda:0")
        for t in range(warm + steps):
            env.gen_actions(t, out=acts[t])
        env.reset()
        row = torch.empty(n, dtype=torch.int32, device="cuda:0")
        for t in range(preroll):
            env.step(env.gen_actions(1_000_000 + t, out=row))
        for t in range(warm):
            env.step(acts[t])
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.synchronize()
        e0.record(s)
        for t in range(steps):
            env.step(acts[warm + t])
        e1.record(s)
        s.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / steps
        mix = {"cargo_gt0": float((env.cargo > 0).float().mean()), "fuel_mean": float(env.fuel.mean())}
        env.close()
    del acts, row
    torch.cuda.empty_cache()
    return us, mix


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=1 << 24)
    a = p.parse_args()
    for rep in range(2):
        for preroll in (0, 1000):
            for side in (False, True):
                us, mix = run(a.n, preroll, side)
                print(json.dumps({"rep": rep, "n": a.n, "preroll": preroll, "own_stream": side,
                                  "us_per_step": round(us, 3), **mix}), flush=True)


if __name__ == "__main__":
    main()
