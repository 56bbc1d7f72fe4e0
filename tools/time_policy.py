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
    p.add_argument("--trace", action="store_true",
                   help="a SHIPENV_X3_TRACE=1 library: per-phase cycle medians of the fp32 policy's 4th tile")
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
    # the same in the policy's visiting order (qpolicy.h OrderRun: each workgroup's chunk of
    # 4096 envs at 2^20, ships at sea first): the share of 32-env tiles that need fc3's second tile
    ordered = float("nan")
    if a.n % 4096 == 0:
        c = at.view(-1, 4096).sort(dim=1, stable=True).values  # False (at sea) first
        ordered = float(c.view(-1, 32).any(1).float().mean())
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(a.launches):
        pol.act(a.eps, 1000 + k, precision=a.precision)
    e1.record()
    torch.cuda.synchronize()
    rec = {"lib": os.path.basename(a.lib or "default"), "precision": a.precision,
           "n": a.n, "preroll": a.preroll, "ms_per_launch": round(e0.elapsed_time(e1) / a.launches, 4),
           "at_port": float(at.float().mean()), "wave32_with_port": float(waves_any),
           "order": os.environ.get("SHIPENV_POLICY_ORDER", "auto"), "wave32_with_port_ordered": ordered}
    if a.trace:
        import ctypes
        import numpy as np
        from shippingenv_amd import _native as N

        buf = np.zeros(4096 * 16, dtype=np.uint64)
        N.lib().se_policy_trace_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        assert N.lib().se_policy_trace_read(buf.ctypes.data, buf.nbytes) == 0
        st = buf.reshape(4096, 16).astype(np.int64)
        last = max(k for k in range(9) if (st[:, k] > 0).any())  # the kernel's last phase stamp
        ok = (st[:, 0] > 0) & (st[:, last] > st[:, 0]) & (st[:, 9] >= st[:, 9].max() - 5000)
        d = np.diff(st[ok][:, :last + 1], axis=1)
        rec["trace_waves"] = int(ok.sum())
        rec["phase_cycles_median"] = [int(x) for x in np.median(d, axis=0)]
        rec["tile_cycles_median"] = int(np.median(st[ok][:, last] - st[ok][:, 0]))
        # stamps 9-11: s_memrealtime (100 MHz, chip-wide) at start, image staged, end; the last
        # launch's waves only (a pre-roll's launches of the other kernel may have left more)
        live = (st[:, 9] > 0) & (st[:, 9] >= st[:, 9].max() - 5000)
        s9, s10, s11 = st[live, 9], st[live, 10], st[live, 11]
        t0 = s9.min()
        rec["us_image_median"] = float(np.median(s10 - s9)) / 100
        if (st[live, 15] > 0).all():  # the fp32 kernel's slot 15: its part of the image built
            rec["us_pack_median"] = float(np.median(st[live, 15] - s9)) / 100
        rec["us_wave_median"] = float(np.median(s11 - s9)) / 100
        rec["us_start_spread_max"] = float((s9 - t0).max()) / 100
        rec["us_end_median"] = float(np.median(s11 - t0)) / 100
        rec["us_end_max"] = float((s11 - t0).max()) / 100
        # stamps 12-14: s_memtime (shader clock) beside 9-11: the wave's mean clock
        rec["ghz_wave_median"] = float(np.median((st[live, 14] - st[live, 12]) / (s11 - s9) / 10))
        wpb = 8 if a.precision == "f32" else 16  # waves per workgroup; the last quarter / half at issue priority 1
        wid = np.nonzero(live)[0] % wpb
        hi = wid >= (4 if wpb == 8 else 12)
        rec["us_wave_median_by_prio"] = [float(np.median((s11 - s9)[~hi])) / 100,
                                         float(np.median((s11 - s9)[hi])) / 100]
        # where the tail is: per XCD (workgroup b on XCD b % 8 under round-robin placement)
        # and per SIMD (wave w of a workgroup on SIMD w % 4), the launch-relative end times
        gw = np.nonzero(live)[0]
        blk, end = gw // wpb, (s11 - t0) / 100
        xcd = blk % 8
        rec["us_end_by_xcd_median"] = [round(float(np.median(end[xcd == k])), 2) for k in range(8)]
        rec["us_end_by_xcd_max"] = [round(float(end[xcd == k].max()), 2) for k in range(8)]
        rec["us_start_by_xcd_median"] = [round(float(np.median((s9 - t0)[xcd == k])) / 100, 2) for k in range(8)]
        simd = blk * 4 + (gw % wpb) % 4
        last = np.zeros(simd.max() + 1)
        np.maximum.at(last, simd, end)
        last = last[np.unique(simd)]
        rec["us_simd_last_end_q"] = [round(float(np.quantile(last, q)), 2) for q in (0.0, 0.1, 0.5, 0.9, 1.0)]
        rec["us_wave_end_q"] = [round(float(np.quantile(end, q)), 2) for q in (0.0, 0.1, 0.5, 0.9, 1.0)]
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
