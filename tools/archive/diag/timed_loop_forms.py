"""Where the driver's short timed region loses wall time outside the kernels (diagnostic):
bench.py's config-3 timed loop (N = 2^20, K = 20 back-to-back steps between a synchronize
on either side) in a few forms, alternated in one process, 30 repetitions each:

  bench      as bench.py: event before launch 1, event after launch 1, event after K
  no_e0      the event before launch 1 dropped (recorded after launch 1 instead)
  evsync     bench, then the last event synchronised (hipEventSynchronize) before the
             device synchronize (which then finds the GPU idle)
  bare       no events at all

    python tools/diag/timed_loop_forms.py
Prints one JSON line: median and min wall us per step of each form.
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

    n, K = 1 << 20, 20
    env = VecEnv(n, seed=2026, device="cuda:0")
    acts = torch.empty((64, n), dtype=torch.int32, device="cuda:0")
    for t in range(64):
        env.gen_actions(t, out=acts[t])
    env.reset()
    rows = [acts[k] for k in range(64)]
    s = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for k in range(50):
        env.step(rows[k % 64])
    torch.cuda.synchronize()

    def run(form, base):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if form in ("bench", "evsync"):
            ev[0].record(s)
        for k in range(K):
            env.step(rows[(base + k) % 64])
            if k == 0 and form != "bare":
                ev[1].record(s)
        if form != "bare":
            ev[2].record(s)
        if form == "evsync":
            ev[2].synchronize()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / K * 1e6

    forms = ("bench", "no_e0", "evsync", "bare")
    res = {f: [] for f in forms}
    for rep in range(30):
        for i, f in enumerate(forms):
            res[f].append(run(f, rep * 7 + i))
    print(json.dumps({f: {"median_us": round(statistics.median(v), 3), "min_us": round(min(v), 3)}
                      for f, v in res.items()}))
    env.close()


if __name__ == "__main__":
    main()
