"""The fused DQN update issued as one HIP graph replay against eager launches (diagnostic):
VecDQNAgent.update() K times back to back at 2^20 envs, B = 8192, after the training loop
has filled the ring; per form, HIP events around the K updates (GPU ms per update), the host
time to issue them (before the synchronize) and the wall time per update.

    python tools/diag/update_forms.py [--iters 50]
One JSON line per form and repetition.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=1 << 20)
    p.add_argument("--batch", type=int, default=8192)
    p.add_argument("--iters", type=int, default=50)
    p.add_argument("--lib", default=None)
    p.add_argument("--forms", default="graph,eager")
    p.add_argument("--device-key", action="store_true",
                   help="eager updates read the sampler key and ring size on the device (t=None)")
    a = p.parse_args()
    if a.lib:
        from shippingenv_amd import _native

        _native.LIB_PATH = os.path.abspath(a.lib)
    from shippingenv_amd.dqn import VecDQNAgent
    from shippingenv_amd.vec import VecEnv

    env = VecEnv(a.n, seed=2026, auto_reset=True, device="cuda:0")
    env.reset()
    torch.manual_seed(2026)
    agent = VecDQNAgent(env, batch_size=a.batch, memory_size=4 * a.n, graph=True)
    if a.device_key:
        step_replay = agent.trainer.step_replay
        agent.trainer.step_replay = lambda *args, t=None, **kw: step_replay(*args, t=None, **kw)
    for _ in range(6):
        agent.step()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    graph = agent._graph
    for rep in range(3):
        for form in a.forms.split(","):
            agent._graph = graph if form == "graph" else None
            agent.use_graph = form == "graph"
            agent.update()  # one untimed
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record(s)
            for _ in range(a.iters):
                agent.update()
            e1.record(s)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            print(json.dumps({"lib": os.path.basename(a.lib or "default"), "device_key": a.device_key,
                              "rep": rep, "form": form, "iters": a.iters,
                              "gpu_ms_per_update": round(e0.elapsed_time(e1) / a.iters, 4),
                              "host_issue_ms_per_update": round((t1 - t0) * 1e3 / a.iters, 4),
                              "wall_ms_per_update": round((t2 - t0) * 1e3 / a.iters, 4)}), flush=True)
    agent._graph = graph
    agent.close()
    env.close()


if __name__ == "__main__":
    main()
