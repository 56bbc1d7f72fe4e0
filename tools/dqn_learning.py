"""Does the vectorised DQN trainer learn? (agents/dqn.py:247-347.)

    python tools/dqn_learning.py --n 65536 --iters 3000 --every 250 --updates-per-step 1

Trains VecDQNAgent with the reference's gamma 0.95, lr 1e-3, batch 32 and epsilon schedule
(1.0, x0.995 per update, floor 0.01; utils/constants.py:21-53) on an auto-reset VecEnv, and
every `every` iterations evaluates the current network greedily (epsilon 0) beside the
epsilon = 1 policy (uniform over the valid actions: the reference's random.choice) on the same
evaluation states, two ways:

* `from_reset`: every ship at its origin port (VecEnv.reset), `--horizon` steps. The return per
  env over that horizon (every env counts; the reference's only `done` is running out of fuel,
  environment.py:296-299, so a greedy ship that stays in port ends no episode).
* `at_sea`: the states after `--preroll` steps of the epsilon = 1 policy from reset (ships
  under way to their destinations, as bench.py's config 5), `--horizon` steps.

Each evaluation env is rebuilt from the same seed, so every row sees the same states. With
--preroll-train the training env starts from the at-sea states too. One JSON line per
evaluation; updates per env-step = updates_per_step / n (the reference takes one update per
single-env step, agents/dqn.py:292).
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def preroll(env, steps, t0=5_000_000):
    """`steps` steps of the epsilon = 1 policy (its choice does not read the weights)."""
    from shippingenv_amd.policy import QPolicy

    pol = QPolicy(env)
    for t in range(steps):
        env.step(pol.act(1.0, t0 + t))
    pol.close()


def evaluate(n, seed, model, eps, horizon, pre, t0):
    """Mean return per env over `horizon` steps of the policy (epsilon `eps`, network `model`)
    from reset (pre = 0) or from the at-sea states after `pre` random steps; the share of the
    evaluation's envs that were at sea at its start; finished episodes."""
    from shippingenv_amd.policy import QPolicy
    from shippingenv_amd.vec import VecEnv

    env = VecEnv(n, seed=seed, device="cuda:0", auto_reset=True)
    env.reset()
    if pre:
        preroll(env, pre)
    px = torch.as_tensor(env.port_x, device=env.device).long()
    py = torch.as_tensor(env.port_y, device=env.device).long()
    at_port = ((env.x.long()[:, None] == px[None]) & (env.y.long()[:, None] == py[None])).any(1)
    env.clear_stats()
    pol = QPolicy(env, model)
    total = torch.zeros(n, dtype=torch.float64, device=env.device)
    for t in range(horizon):
        env.step(pol.act(eps, t0 + t))
        total += env.reward.double()
    st = env.episode_stats().cpu().tolist()
    out = {"return_per_env": float(total.mean()), "reward_per_env_step": float(total.mean()) / horizon,
           "return_at_sea_start": float(total[~at_port].mean()) if bool((~at_port).any()) else None,
           "share_at_sea_start": float((~at_port).double().mean()), "episodes": int(st[1]),
           "mean_episode_return": st[0] / st[1] if st[1] else None}
    pol.close()
    env.close()
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=1 << 16)
    p.add_argument("--iters", type=int, default=3000)
    p.add_argument("--every", type=int, default=250)
    p.add_argument("--updates-per-step", type=int, default=1)
    p.add_argument("--horizon", type=int, default=100)
    p.add_argument("--preroll", type=int, default=300)
    p.add_argument("--preroll-train", action="store_true")
    p.add_argument("--seed", type=int, default=2026)
    p.add_argument("--precision", default="bf16", choices=("bf16", "f32"))
    p.add_argument("--target-update-every", type=int, default=1000)
    p.add_argument("--tag", default="")
    p.add_argument("--torch", action="store_true", help="the torch autograd + Adam update (fused=False)")
    a = p.parse_args()
    from shippingenv_amd.dqn import VecDQNAgent
    from shippingenv_amd.vec import VecEnv

    torch.manual_seed(a.seed)
    env = VecEnv(a.n, seed=a.seed, device="cuda:0", auto_reset=True)
    env.reset()
    if a.preroll_train:
        preroll(env, a.preroll, t0=6_000_000)
    agent = VecDQNAgent(env, updates_per_step=a.updates_per_step, precision=a.precision,
                        target_update_every=a.target_update_every, fused=not a.torch)
    base = {"tag": a.tag, "n": a.n, "updates_per_step": a.updates_per_step,
            "updates_per_env_step": a.updates_per_step / a.n, "precision": a.precision,
            "gamma": agent.gamma, "lr": agent.learning_rate, "batch": agent.batch_size,
            "horizon": a.horizon, "preroll_train": a.preroll_train, "update": "torch" if a.torch else "fused",
            "target_update_every": a.target_update_every}
    es = a.seed + 1
    for where, pre in (("from_reset", 0), ("at_sea", a.preroll)):
        r = evaluate(a.n, es, agent.model, 1.0, a.horizon, pre, 9_000_000)
        print(json.dumps(base | {"eval": where, "policy": "random (epsilon 1)", **r}), flush=True)
    t_start = time.perf_counter()
    for k in range(a.iters + 1):
        if k % a.every == 0:
            loss = float(agent._loss)
            # what the training env is doing: its share of ships in port, and their fuel
            # (take_fuel is unbounded, environment.py:351-357, so fuel grows in port)
            tpx = torch.as_tensor(env.port_x, device=env.device).long()
            tpy = torch.as_tensor(env.port_y, device=env.device).long()
            in_port = ((env.x.long()[:, None] == tpx[None]) & (env.y.long()[:, None] == tpy[None])).any(1)
            train = {"train_share_in_port": float(in_port.double().mean()),
                     "train_fuel_mean": float(env.fuel.mean()), "train_fuel_max": float(env.fuel.max())}
            for where, pre in (("from_reset", 0), ("at_sea", a.preroll)):
                g = evaluate(a.n, es, agent.model, 0.0, a.horizon, pre, 8_000_000)
                print(json.dumps(base | {"eval": where, "policy": "greedy", "iter": k, "env_steps": k * a.n,
                                         "updates": agent.updates, "epsilon": round(agent.epsilon, 4),
                                         "loss": loss, "train_s": round(time.perf_counter() - t_start, 2),
                                         **train, **g}),
                      flush=True)
        if k < a.iters:
            agent.step()
    agent.close()
    env.close()


if __name__ == "__main__":
    main()
