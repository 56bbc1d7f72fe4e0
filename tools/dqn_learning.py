"""Does the vectorised DQN trainer learn? (agents/dqn.py:247-347.)

    python tools/dqn_learning.py --n 65536 --iters 3000 --every 250 --updates-per-step 1

Trains VecDQNAgent (the reference's gamma 0.95, lr 1e-3, batch 32, epsilon 1.0 decaying by
0.995 per update to 0.01; utils/constants.py:21-53) on an auto-reset VecEnv and every `every`
iterations evaluates the current network greedily (epsilon 0) on a separate evaluation env from
reset, `--eval-steps` steps, beside the epsilon = 1 policy (uniform over the valid actions, the
reference's random.choice) on the same evaluation states:

* reward_per_env_step: the mean reward of every env over the evaluation steps (every env
  counts, whether or not its episode ended; the reference's only `done` is running out of
  fuel, environment.py:296-299, so a policy that keeps its ships fuelled ends few episodes);
* episodes / mean_episode_return: the evaluation's finished episodes (se_episode_stats).

One JSON line per evaluation. Updates per env-step: updates_per_step / n (the reference takes
one update per single-env step, agents/dqn.py:292).
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def evaluate(env, model, eps, steps, t0):
    from shippingenv_amd.policy import QPolicy

    env.reset()
    env.clear_stats()
    pol = QPolicy(env, model)
    total = torch.zeros((), dtype=torch.float64, device=env.device)
    for t in range(steps):
        env.step(pol.act(eps, t0 + t))
        total += env.reward.double().sum()
    st = env.episode_stats().cpu().tolist()
    pol.close()
    return {"reward_per_env_step": float(total) / (env.n * steps), "episodes": int(st[1]),
            "mean_episode_return": st[0] / st[1] if st[1] else None}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=1 << 16)
    p.add_argument("--iters", type=int, default=3000)
    p.add_argument("--every", type=int, default=250)
    p.add_argument("--updates-per-step", type=int, default=1)
    p.add_argument("--eval-steps", type=int, default=200)
    p.add_argument("--seed", type=int, default=2026)
    p.add_argument("--precision", default="bf16", choices=("bf16", "f32"))
    p.add_argument("--target-update-every", type=int, default=1000)
    p.add_argument("--tag", default="")
    a = p.parse_args()
    from shippingenv_amd.dqn import VecDQNAgent
    from shippingenv_amd.vec import VecEnv

    torch.manual_seed(a.seed)
    env = VecEnv(a.n, seed=a.seed, device="cuda:0", auto_reset=True)
    env.reset()
    ev = VecEnv(a.n, seed=a.seed + 1, device="cuda:0", auto_reset=True)
    agent = VecDQNAgent(env, updates_per_step=a.updates_per_step, precision=a.precision,
                        target_update_every=a.target_update_every)
    base = {"tag": a.tag, "n": a.n, "updates_per_step": a.updates_per_step,
            "updates_per_env_step": a.updates_per_step / a.n, "precision": a.precision,
            "gamma": agent.gamma, "lr": agent.learning_rate, "batch": agent.batch_size}
    rnd = evaluate(ev, agent.model, 1.0, a.eval_steps, 9_000_000)
    print(json.dumps(base | {"policy": "random (epsilon 1)", **rnd}), flush=True)
    t_start = time.perf_counter()
    for k in range(a.iters + 1):
        if k % a.every == 0:
            loss = float(agent._loss)
            g = evaluate(ev, agent.model, 0.0, a.eval_steps, 8_000_000)
            print(json.dumps(base | {"policy": "greedy", "iter": k, "env_steps": k * a.n,
                                     "updates": agent.updates, "epsilon": round(agent.epsilon, 4),
                                     "loss": loss, "train_s": round(time.perf_counter() - t_start, 2), **g}),
                  flush=True)
        if k < a.iters:
            agent.step()
    agent.close()
    ev.close()
    env.close()


if __name__ == "__main__":
    main()
