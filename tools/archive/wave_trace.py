"""Per-wave phase timeline of one step_kernel launch (diagnostic; needs a build with
-DSHIPENV_TRACE=1, see tools/build_trace.sh). Stamps are s_memrealtime (100 MHz):
0 start, 1 world staged (after the barrier), 2 first group stepped (stores issued),
3 end (stores acknowledged). Prints percentiles in us relative to the first start.

    python tools/wave_trace.py --lib shippingenv_amd/_lib/trace/libshipenv_hip.so [--config 3]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--lib", required=True)
    p.add_argument("--n", type=int, default=1 << 20)
    p.add_argument("--config", type=int, default=3)
    p.add_argument("--steps", type=int, default=30)
    a = p.parse_args()
    from shippingenv_amd import _native

    _native.LIB_PATH = os.path.abspath(a.lib)
    from shippingenv_amd.maps import builtin_water
    from shippingenv_amd.vec import VecEnv, random_water_ports

    ports = random_water_ports(builtin_water(), 64, seed=3) if a.config == 4 else None
    env = VecEnv(a.n, seed=2026, ports=ports, auto_reset=a.config == 4, device="cuda:0")
    acts = torch.empty((a.steps, a.n), dtype=torch.int32, device="cuda:0")
    for t in range(a.steps):
        env.gen_actions(t, out=acts[t])
    env.reset()
    torch.cuda.synchronize()
    for t in range(a.steps):
        env.step(acts[t])
    torch.cuda.synchronize()
    waves = (a.n // 4 + 63) // 64
    buf = np.zeros((1 << 16) * 8, dtype=np.uint64)
    lib = ctypes.CDLL(_native.LIB_PATH)
    assert lib.se_trace_read(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes)) == 0
    half = (1 << 16) // 2
    both = buf.reshape(-1, 8)[:, :4].astype(np.int64)
    last = (a.steps - 1) & 1  # the last step's parity (t counts from the first step after reset)
    allst = buf.reshape(-1, 8).astype(np.int64)
    tr = both[last * half:last * half + waves]
    ex = allst[last * half:last * half + waves, 4:7]
    prev = both[(1 - last) * half:(1 - last) * half + waves]
    t0 = tr[:, 0].min()
    us = (tr - t0) / 100.0  # 100 MHz ticks -> us
    pct = lambda x: [round(float(np.percentile(x, q)), 2) for q in (0, 10, 50, 90, 100)]
    out = {"n": a.n, "config": a.config, "waves": int(waves), "percentiles": "0/10/50/90/100",
           "start": pct(us[:, 0]), "staged": pct(us[:, 1]), "stepped": pct(us[:, 2]), "end": pct(us[:, 3]),
           "stage_dur": pct(us[:, 1] - us[:, 0]), "step_dur": pct(us[:, 2] - us[:, 1]),
           "drain_dur": pct(us[:, 3] - us[:, 2]), "life": pct(us[:, 3] - us[:, 0])}
    if (ex > 0).all():  # agent path stamps: data arrived, first half computed, first stores issued
        ue = (ex - t0) / 100.0
        out.update({"arrived": pct(ue[:, 0]), "half1": pct(ue[:, 1]), "stored1": pct(ue[:, 2]),
                    "wait_data": pct(ue[:, 0] - us[:, 1]), "half1_dur": pct(ue[:, 1] - ue[:, 0]),
                    "draws_stores_dur": pct(ue[:, 2] - ue[:, 1]), "half2_dur": pct(us[:, 2] - ue[:, 2])})
    out["prev_end_to_start_us"] = round(float((t0 - prev[:, 3].max()) / 100.0), 2)
    out["prev_first_start_to_start_us"] = round(float((t0 - prev[:, 0].min()) / 100.0), 2)
    # waves alive over time (10 bins per us)
    edges = np.arange(0, us[:, 3].max() + 0.1, 0.5)
    alive = [int(((us[:, 0] <= e) & (us[:, 3] > e)).sum()) for e in edges]
    out["alive_every_0.5us"] = alive
    env.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
