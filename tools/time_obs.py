"""Time the observation gather (se_observe: preprocess_state rows), the DQN validity
mask (se_valid_mask) and the random policy (se_sample_actions) at N envs, against the
HBM bytes each writes.

    python tools/time_obs.py [--n N] [--ports 5|64] [--reps K] [--lib path]
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
    p.add_argument("--ports", type=int, default=5)
    p.add_argument("--reps", type=int, default=50)
    p.add_argument("--lib", default=None)
    a = p.parse_args()
    if a.lib:
        from shippingenv_amd import _native

        _native.LIB_PATH = os.path.abspath(a.lib)
    from shippingenv_amd.maps import builtin_water
    from shippingenv_amd.vec import VecEnv, random_water_ports

    ports = random_water_ports(builtin_water(), 64, seed=3) if a.ports == 64 else None
    env = VecEnv(a.n, seed=2026, ports=ports, device="cuda:0")
    env.reset()
    for t in range(5):
        env.step(env.gen_actions(t))
    obs = env.observe()
    bits = env.valid_mask()
    smp = env.sample_actions(7)
    s = torch.cuda.current_stream()
    out = {"lib": os.path.basename(a.lib or "default"), "n": a.n, "P": env.P}
    for name, fn, nbytes in (("observe", lambda: env.observe(obs), obs.numel() * 4),
                             ("valid_mask", lambda: env.valid_mask(bits), bits.numel()),
                             ("sample_actions", lambda: env.sample_actions(7, smp), 12 * env.n)):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.reps):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / a.reps * 1e3
        out[name + "_us"] = round(us, 2)
        out[name + "_write_TBps"] = round(nbytes / (us * 1e-6) / 1e12, 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
