"""Phase timeline of the DQN update's T1 kernel (diagnostic; needs a build with
-DSHIPENV_QTRACE=1): s_memrealtime (100 MHz) stamps per wave at kernel start and after
each of its barriers (1 inputs staged, 2 fc1, 3 fc2, 4 target fc3 + max, 5 targets y,
6 q and g, 7 dZ2, 8 dH1 / dW2 / dW3), then 9 at the end, and 14 / 15 when a wave's own fc2 /
fc3 chain is done (before the phase's barrier). Runs a few training steps and prints, for the
last T1 launch, per-phase medians over workgroups (us), the launch span and each wave's fc2 /
fc3 completion; T2's stamps (slots 10-13) per block kind.

    bash -c 'hipcc ... -DSHIPENV_QTRACE=1 -o /tmp/qt.so ...'; python tools/qtrain_trace.py --lib /tmp/qt.so
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
    p.add_argument("--batch", type=int, default=8192)
    p.add_argument("--inputs", action="store_true",
                   help="a SHIPENV_QTRACE=2 build: slots 14 / 15 are wave 0's picks issued / in LDS")
    a = p.parse_args()
    from shippingenv_amd import _native

    _native.LIB_PATH = os.path.abspath(a.lib)
    from shippingenv_amd.dqn import VecDQNAgent
    from shippingenv_amd.vec import VecEnv

    env = VecEnv(a.n, seed=2026, auto_reset=True, device="cuda:0")
    env.reset()
    torch.manual_seed(2026)
    agent = VecDQNAgent(env, batch_size=a.batch, memory_size=4 * a.n, graph=False)
    for _ in range(8):
        agent.step()
    torch.cuda.synchronize()
    wg, stamps = 1024, 16
    buf = np.zeros(wg * 8 * stamps, np.uint64)
    lib = ctypes.CDLL(_native.LIB_PATH)
    assert lib.se_qtrace_read(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes)) == 0
    tiles = (a.batch + 31) // 32
    t = buf.reshape(wg, 8, stamps)[:tiles, :, :10].astype(np.int64)
    t0 = t[:, :, 0].min()
    rel = (t - t0) / 100.0  # 100 MHz -> us
    wgmax = rel.max(axis=1)  # per workgroup: the slowest wave at each stamp
    out = {"tiles": tiles, "span_us": float(rel[:, :, 9].max()),
           "wg_alone_median_us": float(np.median(wgmax[:, 9] - rel[:, :, 0].min(axis=1)))}
    phases = ["start", "inputs", "fc1", "fc2", "fc3_max", "targets", "q_g", "dZ2", "dH1_dW2_dW3", "end"]
    d = np.diff(wgmax, axis=1)
    out["phase_median_us"] = {phases[k + 1]: round(float(np.median(d[:, k])), 3) for k in range(9)}
    out["start_spread_us"] = float(np.percentile(rel[:, :, 0].min(axis=1), 99))
    # T2 (slots 10-13, 4 waves): W1 rows [0, 128), W2 blocks [128, 384), then one block per
    # W3 row (mt3 x 32 rows, b3 with its row)
    nb = 384 + int(os.environ.get("QT_W3_BLOCKS_PER_ROW", "2")) * 32 * ((4 + int(env.P) + 250 + 31) // 32)
    t2 = buf.reshape(wg, 8, stamps)[:nb, :4, 10:14].astype(np.int64)
    t20 = t2[:, :, 0].min()
    r2 = (t2 - t20) / 100.0
    w2 = r2.max(axis=1)
    out["t2_span_us"] = float(r2[:, :, 3].max())
    out["t2_gap_after_t1_us"] = float((t20 - t[:, :, 9].max()) / 100.0)
    for name, lo, hi in (("w1", 0, 128), ("w2", 128, 384), ("w3", 384, nb)):
        d2 = np.diff(w2[lo:hi], axis=1)
        out["t2_" + name] = {"start_p50": float(np.median(w2[lo:hi, 0])), "start_max": float(w2[lo:hi, 0].max()),
                             "wsum": float(np.median(d2[:, 0])), "sum": float(np.median(d2[:, 1])),
                             "adam": float(np.median(d2[:, 2])), "end_max": float(w2[lo:hi, 3].max())}
    if a.inputs:  # wave 0 of each T1 workgroup, from its own start (slot 0)
        w0 = buf.reshape(wg, 8, stamps)[:tiles, 0, :].astype(np.int64)
        rel0 = (w0 - w0[:, :1]) / 100.0
        out["inputs_wave0_median_us"] = {"picks_issued": float(np.median(rel0[:, 14])),
                                         "picks_in_lds": float(np.median(rel0[:, 15])),
                                         "barrier_passed": float(np.median(rel0[:, 1]))}
        print(json.dumps(out))
        agent.close()
        env.close()
        return
    # slots 14 / 15: each wave's fc2 / fc3 chain done (before the phase's barrier), from the
    # phase start (the slowest wave's stamp after the previous barrier), per wave of a workgroup
    raw = buf.reshape(wg, 8, stamps)[:tiles].astype(np.int64)
    for name, s_end, s0 in (("fc2", 14, 2), ("fc3", 15, 3)):
        d_w = (raw[:, :, s_end] - raw[:, :, s0].max(axis=1, keepdims=True)) / 100.0
        out[name + "_wave_done_median_us"] = [round(float(np.median(d_w[:, k])), 2) for k in range(8)]
    print(json.dumps(out))
    agent.close()
    env.close()


if __name__ == "__main__":
    main()
