"""Separate the state mix from GPU warm-up in the driver's short run.

The driver times 20 steps after 5 warm-up steps from reset; long runs time ~8.5 us per
step. Two things differ between them: the env states (fresh from reset: ships at ports,
TAKE actions valid, cargo rising) and how long the GPU has been stepping. This script
crosses the two, each case in a FRESH process (run it once per case):

    python tools/diag/state_vs_warmup.py --save /tmp/s1000.pt        # 1000 steps, save state
    python tools/diag/state_vs_warmup.py --case reset_cold           # reset, 5 + 20 (the driver)
    python tools/diag/state_vs_warmup.py --case steady_cold --load /tmp/s1000.pt
    python tools/diag/state_vs_warmup.py --case reset_warm           # 1000 steps of another env first
    python tools/diag/state_vs_warmup.py --case steady_warm --load /tmp/s1000.pt

Each prints one JSON line: the wall time per step, the first launch from before its
enqueue (its idle-queue start included), the back-to-back launches 2..20 (HIP events),
and the state mix (envs at a port, cargo > 0).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

FIELDS = ("x", "y", "fuel", "cargo", "origin", "dest")


def make_env(n):
    from shippingenv_amd.vec import VecEnv

    return VecEnv(n, seed=2026, device="cuda:0")


def run_steps(env, steps, t0):
    row = torch.empty(env.n, dtype=torch.int32, device=env.device)
    for t in range(steps):
        env.step(env.gen_actions(t0 + t, out=row))


def mix(env):
    pos = env.x.long() * env.W + env.y.long()
    port_cells = torch.as_tensor(env.port_x * env.W + env.port_y, device=env.device).long()
    at_port = torch.isin(pos, port_cells)
    return {"at_port": round(float(at_port.float().mean()), 4),
            "cargo_gt0": round(float((env.cargo > 0).float().mean()), 4),
            "mean_cargo": round(float(env.cargo.float().mean()), 3),
            "mean_fuel": round(float(env.fuel.mean()), 2)}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=1 << 20)
    p.add_argument("--save")
    p.add_argument("--load")
    p.add_argument("--case", default="reset_cold")
    a = p.parse_args()
    if a.save:
        env = make_env(a.n)
        env.reset()
        run_steps(env, 1000, 500_000)
        torch.cuda.synchronize()
        torch.save({k: getattr(env, k).cpu() for k in FIELDS}, a.save)
        print(json.dumps({"saved": a.save, "mix": mix(env)}))
        return
    if a.case.endswith("_warm"):  # the GPU steps 1000 times before the measured env exists
        w = make_env(a.n)
        w.reset()
        run_steps(w, 1000, 700_000)
        torch.cuda.synchronize()
        w.close()
    env = make_env(a.n)
    acts = torch.empty((25, env.n), dtype=torch.int32, device=env.device)
    for t in range(25):
        env.gen_actions(t, out=acts[t])
    env.reset()
    if a.load:
        saved = torch.load(a.load, weights_only=True)
        for k in FIELDS:
            getattr(env, k).copy_(saved[k])
    m0 = mix(env)
    for k in range(5):
        env.step(acts[k])
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    # as bench.py times it: events only around the launches (an event between every two
    # launches breaks the back-to-back dispatch and adds ~2.5 us per launch)
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    rows = [acts[5 + k] for k in range(20)]
    t0 = time.perf_counter()
    e0.record(s)
    for k in range(20):
        env.step(rows[k])
        if k == 0:
            e1.record(s)
    e2.record(s)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / 20 * 1e6
    print(json.dumps({"case": a.case, "n": a.n, "wall_us_per_step": round(wall, 3),
                      "first_launch_incl_start_us": round(e0.elapsed_time(e1) * 1e3, 3),
                      "back_to_back_us": round(e1.elapsed_time(e2) * 1e3 / 19, 3),
                      "mix_before": m0, "env": {k: os.environ.get(k) for k in ("ROC_ACTIVE_WAIT_TIMEOUT",)}}))


if __name__ == "__main__":
    main()
