"""Host-side cost of VecEnv.step at N = 2^20 (diagnostic): per-call host time with the
queue running, and the wall time of the driver's short timed region (20 steps bracketed
by synchronize) with the action rows indexed per step or sliced beforehand."""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from shippingenv_amd.vec import VecEnv

    n, K = 1 << 20, 200
    env = VecEnv(n, seed=1, device="cuda:0")
    acts = torch.empty((K, n), dtype=torch.int32, device="cuda:0")
    for t in range(K):
        env.gen_actions(t, out=acts[t])
    env.reset()
    for k in range(50):
        env.step(acts[k % K])
    torch.cuda.synchronize()
    out = {}
    t0 = time.perf_counter()
    for k in range(K):
        env.step(acts[k])
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out["host_us_per_call_indexed"] = round((t1 - t0) / K * 1e6, 2)
    out["wall_us_per_step_200"] = round((t2 - t0) / K * 1e6, 2)
    rows = [acts[k] for k in range(K)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        env.step(rows[k])
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    out["host_us_per_call_presliced"] = round((t1 - t0) / K * 1e6, 2)
    s = torch.cuda.current_stream()
    for name, pre in (("indexed", False), ("presliced", True)):
        walls, evs = [], []
        for rep in range(12):
            base = (rep * 20) % (K - 20)
            r = rows[base:base + 20] if pre else None
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record(s)
            if pre:
                for a in r:
                    env.step(a)
            else:
                for k in range(20):
                    env.step(acts[base + k])
            e1.record(s)
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) / 20 * 1e6)
            evs.append(e0.elapsed_time(e1) / 20 * 1e3)
        out[f"short20_{name}_wall_us"] = round(statistics.median(walls), 2)
        out[f"short20_{name}_event_us"] = round(statistics.median(evs), 2)
    # the fixed cost of an empty timed region
    e0 = torch.cuda.Event(enable_timing=True)
    walls = []
    for _ in range(20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(s)
        torch.cuda.synchronize()
        walls.append((time.perf_counter() - t0) * 1e6)
    out["empty_region_us"] = round(statistics.median(walls), 2)
    env.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
