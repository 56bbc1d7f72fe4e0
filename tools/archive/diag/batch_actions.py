"""Histogram of the actions in DQN training minibatches (how skewed the per-action dW3
segments are), after K training iterations at the bench's shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from shippingenv_amd.dqn import VecDQNAgent
    from shippingenv_amd.vec import VecEnv

    env = VecEnv(1 << 20, seed=2026, auto_reset=True, device="cuda:0")
    env.reset()
    torch.manual_seed(2026)
    agent = VecDQNAgent(env, batch_size=8192, memory_size=4 << 20, graph=False)
    for it in range(60):
        agent.step()
        if it in (5, 20, 59):
            torch.cuda.synchronize()
            c = torch.bincount(agent.batch.act, minlength=agent.trainer.q.A if hasattr(agent, "trainer") and hasattr(agent.trainer, "q") else 1)
            top = torch.sort(c, descending=True).values[:8].tolist()
            print(json.dumps({"iter": it, "distinct": int((c > 0).sum()), "top8": top,
                              "tiles_spanned_by_top": [t // 32 + 1 for t in top[:3]]}))
    agent.close()
    env.close()


if __name__ == "__main__":
    main()
