"""Step-loop launch path comparison (diagnostic): K steps launched from Python
(VecEnv.step per step) against the same K steps captured in one HIP graph and
replayed. The graph bakes each node's step counter, so replays repeat the draws:
timing only.

    python tools/time_graph.py [--n N] [--config 3|4] [--steps K]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=1 << 20)
    p.add_argument("--config", type=int, default=3)
    p.add_argument("--steps", type=int, default=200)
    a = p.parse_args()
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
    py = (time.perf_counter() - t0) / a.steps * 1e6
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for t in range(a.steps):
                env.step(acts[t])
    g.replay()
    torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    gr = (time.perf_counter() - t0) / (reps * a.steps) * 1e6
    env.close()
    print(json.dumps({"n": a.n, "config": a.config, "python_loop_us": round(py, 2), "graph_us": round(gr, 2)}))


if __name__ == "__main__":
    main()
