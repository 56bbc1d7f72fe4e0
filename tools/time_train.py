"""Time the parts of one vectorised DQN training iteration (shippingenv_amd.dqn) on one GPU.

    python tools/time_train.py [--n N] [--batch B] [--iters K] [--eager]

Prints one JSON line: HIP-event ms per iteration of each part on the launch stream
(the fused launches VecDQNAgent.step makes: policy + begin, step + end + reset; with --pair the
step and the end + reset as two launches; with --separate the policy, replay begin, step, replay
end and reset of cut envs), the update, and the whole loop.
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
    p.add_argument("--batch", type=int, default=8192)
    p.add_argument("--iters", type=int, default=30)
    p.add_argument("--eager", action="store_true", help="no graph capture of the update")
    p.add_argument("--lib", default=None)
    p.add_argument("--separate", action="store_true",
                   help="time the separate launches (policy, begin, step, end, reset) instead of the "
                        "fused ones VecDQNAgent.step uses (policy + begin, step, end + reset)")
    p.add_argument("--pair", action="store_true",
                   help="the step and the replay end + reset as two launches (se_step, se_replay_end_reset)")
    a = p.parse_args()
    if a.lib:
        from shippingenv_amd import _native

        _native.LIB_PATH = os.path.abspath(a.lib)
    from shippingenv_amd.dqn import VecDQNAgent
    from shippingenv_amd.vec import VecEnv

    env = VecEnv(a.n, seed=2026, auto_reset=True, device="cuda:0")
    env.reset()
    torch.manual_seed(2026)
    agent = VecDQNAgent(env, batch_size=a.batch, memory_size=4 * a.n, graph=False if a.eager else None)
    for _ in range(6):
        agent.step()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    parts = ("policy", "begin", "step", "end", "reset", "update") if a.separate else \
        ("policy_record", "step", "end_reset", "update") if a.pair else ("policy_record", "step_record", "update")
    ev = {k: [] for k in parts}

    def mark(name, fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        r = fn()
        e1.record(s)
        ev[name].append((e0, e1))
        return r

    g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g0.record(s)
    for _ in range(a.iters):
        if a.separate:
            act = mark("policy", agent.choose_actions)
            mark("begin", lambda: agent.memory.begin(act))
            mark("step", lambda: env.step(act))
            mark("end", lambda: agent.memory.end(agent.cut, agent.max_steps))
            mark("reset", lambda: env.reset(agent.cut))
        elif a.pair:
            act = mark("policy_record", lambda: agent.policy.act_record(agent.memory, agent.epsilon, agent.t))
            mark("step", lambda: env.step(act))
            mark("end_reset", lambda: agent.memory.end(agent.cut, agent.max_steps, reset=True))
        else:
            act = mark("policy_record", lambda: agent.policy.act_record(agent.memory, agent.epsilon, agent.t))
            mark("step_record", lambda: agent.memory.step_end(act, agent.cut, agent.max_steps))
        mark("update", agent.update)
        agent.t += 1
    g1.record(s)
    torch.cuda.synchronize()
    mode = "separate" if a.separate else "pair" if a.pair else "fused"
    out = {"lib": os.path.basename(a.lib or "default"), "mode": mode, "n": a.n, "batch": a.batch, "graph": not a.eager,
           "loop_ms": round(g0.elapsed_time(g1) / a.iters, 4)}
    for k in parts:
        out[k + "_ms"] = round(sum(x.elapsed_time(y) for x, y in ev[k]) / a.iters, 4)
    agent.close()
    env.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
