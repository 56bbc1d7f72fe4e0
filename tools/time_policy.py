"""Time the fused DQN policy step (se_policy) on one GPU and report the share of
envs at a port (whose rows beyond the 4 moves can be valid).

    python tools/time_policy.py [--n N] [--launches K] [--steps S]
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
    p.add_argument("--launches", type=int, default=20)
    p.add_argument("--steps", type=int, default=20, help="policy+step iterations before timing")
    p.add_argument("--preroll", type=int, default=0,
                   help="bench.py config 5's state: auto-reset envs, this many steps at epsilon 1.0 "
                        "(bench: 300) before the --steps ones")
    p.add_argument("--eps", type=float, default=0.1)
    p.add_argument("--lib", default=None)
    p.add_argument("--precision", default="bf16", choices=("bf16", "f32"))
    a = p.parse_args()
    if a.lib:
        from shippingenv_amd import _native

        _native.LIB_PATH = os.path.abspath(a.lib)
    from shippingenv_amd.policy import DQNNetwork, QPolicy
    from shippingenv_amd.vec import VecEnv

    env = VecEnv(a.n, seed=2026, device="cuda:0", auto_reset=a.preroll > 0)
    env.reset()
    torch.manual_seed(2026)
    pol = QPolicy(env, DQNNetwork(env.obs_size, env.action_space_size))
    for t in range(a.preroll):
        env.step(pol.act(1.0, 200_000 + t))
    for t in range(a.steps):
        env.step(pol.act(a.eps, t))
    px = torch.as_tensor(env.port_x, device="cuda:0").long()
    py = torch.as_tensor(env.port_y, device="cuda:0").long()
    at = ((env.x.long()[:, None] == px[None]) & (env.y.long()[:, None] == py[None])).any(1)
    waves_any = at.view(-1, 32).any(1).float().mean() if a.n % 32 == 0 else float("nan")
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(a.launches):
        pol.act(a.eps, 1000 + k, precision=a.precision)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"lib": os.path.basename(a.lib or "default"), "precision": a.precision,
                      "n": a.n, "preroll": a.preroll, "ms_per_launch": round(e0.elapsed_time(e1) / a.launches, 4),
                      "at_port": float(at.float().mean()), "wave32_with_port": float(waves_any)}))


if __name__ == "__main__":
    main()
