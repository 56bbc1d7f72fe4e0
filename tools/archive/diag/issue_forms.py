"""Config 3's timed region issued two ways, alternated in one process (diagnostic):
bench.py's timed_loop with VecEnv.step_seq (native launch loop) and with one VecEnv.step
per step from Python, on one N = 2^20 env set after a 1000-step pre-roll; `reps` rounds
of K = 20 steps each, the two forms alternating, so clock or state drift over the process
affects both alike.

    python tools/diag/issue_forms.py [--reps 15]
Prints one JSON line per form: median / min of wall us per step and of the events
basis (end of launch 1 to end of launch K over K - 1), and the per-rep lists.
"""
import argparse
import importlib.util
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=15)
    p.add_argument("--steps", type=int, default=20)
    a = p.parse_args()
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    from shippingenv_amd.vec import VecEnv

    dist = b.Dist(1)
    n, K = 1 << 20, a.steps
    env = VecEnv(n, seed=2026, device=dist.dev)
    acts = b.make_actions(env, 64 + K)
    env.reset()
    row = torch.empty(n, dtype=torch.int32, device=env.device)
    for t in range(1000):
        env.step(env.gen_actions(1_000_000 + t, out=row))
    torch.cuda.synchronize()
    res = {"step_seq": {"wall": [], "events": []}, "per_call": {"wall": [], "events": []}}
    for rep in range(a.reps):
        for form in ("step_seq", "per_call") if rep % 2 == 0 else ("per_call", "step_seq"):
            wall, k_ms = b.timed_loop(env, acts, (rep * 3) % 64, K, dist, step_seq=form == "step_seq")
            res[form]["wall"].append(round(wall / K * 1e6, 3))
            res[form]["events"].append(round(k_ms * 1e3, 3))
    for form, r in res.items():
        print(json.dumps({"form": form, "wall_us_median": statistics.median(r["wall"]),
                          "wall_us_min": min(r["wall"]), "events_us_median": statistics.median(r["events"]),
                          "events_us_min": min(r["events"]), **r}))
    env.close()
    dist.close()


if __name__ == "__main__":
    main()
