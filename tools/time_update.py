"""Back-to-back DQN updates (VecDQNAgent.update, the fused two-launch path) on one GPU:
HIP-event ms per update on the stream, and the host's issue time per update (the loop timed
without a sync, so a host-bound loop shows issue time >= event time).

    python tools/time_update.py [--lib L] [--updates K] [--graph]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=1 << 20)
    p.add_argument("--batch", type=int, default=8192)
    p.add_argument("--updates", type=int, default=200)
    p.add_argument("--graph", action="store_true")
    p.add_argument("--lib", default=None)
    a = p.parse_args()
    if a.lib:
        from shippingenv_amd import _native

        _native.LIB_PATH = os.path.abspath(a.lib)
    from shippingenv_amd.dqn import VecDQNAgent
    from shippingenv_amd.vec import VecEnv

    env = VecEnv(a.n, seed=2026, auto_reset=True, device="cuda:0")
    env.reset()
    torch.manual_seed(2026)
    agent = VecDQNAgent(env, batch_size=a.batch, memory_size=4 * a.n, graph=None if a.graph else False)
    for _ in range(8):
        agent.step()
    for _ in range(20):
        agent.update()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    h0 = time.perf_counter()
    for _ in range(a.updates):
        agent.update()
    h1 = time.perf_counter()
    e1.record(s)
    torch.cuda.synchronize()
    print(json.dumps({"lib": os.path.basename(a.lib or "product"), "graph": a.graph, "updates": a.updates,
                      "update_ms": round(e0.elapsed_time(e1) / a.updates, 5),
                      "host_issue_ms": round((h1 - h0) * 1e3 / a.updates, 5),
                      "target_update_every": agent.target_update_every}))
    agent.close()
    env.close()


if __name__ == "__main__":
    main()
