"""Step-kernel throughput and HBM-roofline fraction against the number of envs.

    python tools/size_sweep.py [--out gpurun_out/size_sweep.json]

For each (N, config): K back-to-back se_step launches over action rows resident in HBM
(the bench's synthetic agent), timed by wall clock between synchronizes, as bench.py
does. frac = algorithmic bytes (42 B per env-step for config 3, 50 B for config 4 (58 before round 5);
DESIGN.md section 3) x N / time per step / 8 TB/s. It shows the regimes of DESIGN.md
section 5: launch-bound below ~2^18, VALU-issue- and launch-bound while the working
set sits in the 256 MiB Infinity Cache (N <= 2^21), HBM-bound beyond.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BYTES = {3: 42, 4: 50}
PEAK = 8000.0  # GB/s, MI355X HBM3E


def one(n, config, steps, preroll=0):
    from shippingenv_amd.maps import builtin_water
    from shippingenv_amd.vec import VecEnv, random_water_ports

    ports = random_water_ports(builtin_water(), 64, seed=3) if config == 4 else None
    env = VecEnv(n, seed=2026, ports=ports, auto_reset=config == 4, device="cuda:0")
    rows = min(steps, 64)  # reuse 64 action rows at the largest sizes (still HBM-resident)
    acts = torch.empty((rows, n), dtype=torch.int32, device="cuda:0")
    for t in range(rows):
        env.gen_actions(t, out=acts[t])
    env.reset()
    row = torch.empty(n, dtype=torch.int32, device="cuda:0")
    for t in range(preroll):  # the bench's steady state: untimed steps from reset, rows of their own
        env.step(env.gen_actions(1_000_000 + t, out=row))
    del row
    for t in range(10):
        env.step(acts[t % rows])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(steps):
        env.step(acts[t % rows])
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / steps * 1e6
    env.close()
    del acts
    torch.cuda.empty_cache()
    gbps = BYTES[config] * n / (us * 1e-6) / 1e9
    return {"n": n, "config": config, "steps": steps, "preroll": preroll, "us_per_step": round(us, 3),
            "env_steps_per_s": round(n / (us * 1e-6), 1), "achieved_gbps": round(gbps, 1),
            "frac": round(gbps / PEAK, 4), "bytes_per_env_step": BYTES[config]}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "size_sweep.json"))
    p.add_argument("--log2n", default="14-25", help="config-3 sizes: a range lo-hi or a list a,b")
    p.add_argument("--log2n4", default="18,20,22,24", help="config-4 sizes ('' = none)")
    p.add_argument("--preroll", type=int, default=1000,
                   help="untimed steps from reset before timing (bench.py's steady state; 0 = from reset)")
    a = p.parse_args()

    def sizes(spec):
        if not spec:
            return []
        if "-" in spec:
            lo, hi = spec.split("-")
            return list(range(int(lo), int(hi) + 1))
        return [int(k) for k in spec.split(",")]

    runs = [(1 << k, 3) for k in sizes(a.log2n)] + [(1 << k, 4) for k in sizes(a.log2n4)]
    res = []
    for n, c in runs:
        steps = 1000 if n <= (1 << 20) else max(50, (1000 << 20) // n)
        r = one(n, c, steps, a.preroll)
        print(json.dumps(r), flush=True)
        res.append(r)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump({"device": torch.cuda.get_device_name(0), "preroll": a.preroll,
                   "nt_loads_env": os.environ.get("SHIPENV_NT_LOADS"), "runs": res}, f, indent=1)


if __name__ == "__main__":
    main()
