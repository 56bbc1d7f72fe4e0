"""How the host waits for the end of the driver's short timed region (diagnostic): bench.py's
config-3 timed loop (N = 2^20, K = 20 steps between a synchronize on either side), issued one
VecEnv.step per step (py) or by the native launch loop VecEnv.step_seq (seq), ended by

  sync   torch.cuda.synchronize() (the runtime's blocking wait)
  spin   polling the last event with query() until it completes, then the synchronize

alternated in one process, 30 repetitions each, from a steady-state (1000-step) env.
Hypothesis under test: a long blocking wait sleeps and wakes late, which the native loop
(all launches issued in ~40 us, then ~130 us of waiting) pays more than the Python loop.

    python tools/diag/wait_forms.py
Prints one JSON line: per form, median / min wall us per step and the events' us per launch.
"""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from shippingenv_amd.vec import VecEnv

    n, K, R = 1 << 20, 20, 64
    env = VecEnv(n, seed=2026, device="cuda:0")
    acts = torch.empty((R, n), dtype=torch.int32, device="cuda:0")
    for t in range(R):
        env.gen_actions(t, out=acts[t])
    env.reset()
    row = torch.empty(n, dtype=torch.int32, device="cuda:0")
    for t in range(1000):
        env.step(env.gen_actions(1_000_000 + t, out=row))
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    ef, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def run(form, base):
        issue, wait = form.split("_")
        b = base % (R - K)
        rows = [acts[b + k] for k in range(K)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if issue == "py":
            env.step(rows[0])
            ef.record(s)
            for k in range(1, K):
                env.step(rows[k])
        else:
            env.step_seq(acts[b:b + 1])
            ef.record(s)
            env.step_seq(acts[b + 1:b + K])
        e1.record(s)
        if wait == "spin":
            while not e1.query():
                pass
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / K * 1e6
        return wall, ef.elapsed_time(e1) * 1e3 / (K - 1)

    forms = ("py_sync", "py_spin", "seq_sync", "seq_spin")
    res = {f: [] for f in forms}
    ker = {f: [] for f in forms}
    for rep in range(30):
        for i, f in enumerate(forms):
            w, k = run(f, rep * 5 + i)
            res[f].append(w)
            ker[f].append(k)
    print(json.dumps({f: {"wall_median_us": round(statistics.median(res[f]), 3), "wall_min_us": round(min(res[f]), 3),
                          "kernel_median_us": round(statistics.median(ker[f]), 3)} for f in forms}))
    env.close()


if __name__ == "__main__":
    main()
