"""Run one of the reference's own agents (agents/dqn.py, sarsa.py, mcts.py, unchanged)
against either the reference's `shipping` package or this repo's drop-in, and print
what it produced as one JSON line.

TEST INFRASTRUCTURE, build container only: it imports the reference's agents and
utils from /root/reference (which never travels to the GPU box), so
tests/test_agent_compat.py skips without it. With the drop-in, state transitions run
through its default stepper, the product's host build of the step kernels' per-env code
(se_host_step_replay; no GPU is needed). tests/test_compat_gpu.py pins that build to the
HIP kernel bit for bit.

    python tests/agent_compat.py --env ref|ours --agent dqn|sarsa|mcts [--seed S]

One process per run: the two `shipping` packages share a module name.
"""
import argparse
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
REF = "/root/reference"


def setup(which):
    if which == "ref":
        sys.path.insert(0, os.path.join(HERE, "golden", "cv2stub"))  # opencv is not installed
        sys.path.insert(0, REF)
    else:
        sys.path.insert(0, REF)  # agents/ and utils/ only: `shipping` resolves to the drop-in
        sys.path.insert(0, os.path.join(ROOT, "shippingenv_amd", "dropin"))
        sys.path.insert(0, ROOT)
        sys.path.insert(0, HERE)
        # the drop-in's default stepper: the product's host build of the step code
        # (SHIPENV_STEPPER=gpu in the environment runs the kernel instead)
    import shipping

    where = os.path.dirname(os.path.abspath(shipping.__file__))
    assert where.startswith(REF if which == "ref" else ROOT), where


def make_env():
    from shipping import Environment
    from utils.constants import DEFAULT_PORTS

    env = Environment("mapa_mundi_binario.jpg")  # cwd is the reference root (agents/mcts.py:190)
    for p in DEFAULT_PORTS:  # main.create_environment (main.py:23-36)
        env.add_port(p)
    return env


def digest(obj):
    return hashlib.sha256(json.dumps(obj, sort_keys=True).encode()).hexdigest()[:16]


def result_dict(res):
    return {"rewards": [float(r) for r in res.episode_rewards],
            "lengths": [int(v) for v in res.episode_lengths],
            "losses": [float(v) for v in res.losses],
            "epsilon": [float(v) for v in res.epsilon_values]}


def run_dqn(seed):
    import numpy as np
    import torch

    from agents.dqn import DQNAgent

    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.use_deterministic_algorithms(True)
    env = make_env()
    agent = DQNAgent(env, batch_size=16)
    res = agent.train(episodes=4, verbose=False, max_steps=60)
    w = torch.cat([p.detach().flatten() for p in agent.model.parameters()]).double()
    return {**result_dict(res), "weights_sum": float(w.sum()), "weights_abs": float(w.abs().sum())}


def run_sarsa(seed):
    import numpy as np

    from agents.sarsa import SARSAAgent

    random.seed(seed)
    np.random.seed(seed)
    env = make_env()
    agent = SARSAAgent(env)
    agent.test_policy = lambda *a, **k: {}  # defect 8: test_policy has no step cap
    res = agent.train(episodes=3, verbose=False, max_total_steps=400)
    q = sorted((repr(k), float(v)) for k, v in agent.q_table.items())
    return {**result_dict(res), "q_entries": len(q), "q_digest": digest(q)}


def run_mcts(seed):
    import numpy as np

    from agents.mcts import MCTSAgent

    random.seed(seed)
    np.random.seed(seed)
    env = make_env()
    agent = MCTSAgent(env, num_simulations=4, max_rollout_steps=20)
    res = agent.train(episodes=2, verbose=False, max_steps=10)
    return result_dict(res)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", choices=("ref", "ours"), required=True)
    ap.add_argument("--agent", choices=("dqn", "sarsa", "mcts"), required=True)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    setup(a.env)
    out = {"dqn": run_dqn, "sarsa": run_sarsa, "mcts": run_mcts}[a.agent](a.seed)
    out["random_after"] = random.random()  # the global stream the env and the agent share
    print("AGENT_COMPAT " + json.dumps(out, sort_keys=True))


if __name__ == "__main__":
    main()
