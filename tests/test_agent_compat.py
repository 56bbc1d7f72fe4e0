"""The reference's own agents (agents/dqn.py, sarsa.py, mcts.py), unchanged, trained
against the reference's `shipping` and against the drop-in under the same seeds give
identical results: episode rewards and lengths, DQN losses and final weights, the SARSA
Q-table, MCTS returns, and the global `random` stream left behind (BASELINE north star:
"agents/{dqn,sarsa,mcts}.py run against it unchanged"; SURVEY §4 agent-compat).

Build container only: the reference never travels to the GPU box. Each run is its own
process (tests/agent_compat.py) because both packages are named `shipping`; the
drop-in's transitions run through its default host stepper (the product's own step code
built for the host), so no GPU is needed."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

REF = "/root/reference"
pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "agents")),
                                reason="needs the reference checkout (build container only)")


def run(env, agent, seed):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "agent_compat.py"), "--env", env,
                        "--agent", agent, "--seed", str(seed)], cwd=REF, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("AGENT_COMPAT ")][-1]
    return json.loads(line[len("AGENT_COMPAT "):])


@pytest.mark.parametrize("agent,seed", [("dqn", 0), ("dqn", 1), ("sarsa", 0), ("mcts", 0)])
def test_reference_agent_runs_identically_on_the_dropin(agent, seed):
    want = run("ref", agent, seed)
    got = run("ours", agent, seed)
    assert got == want
    assert len(want["rewards"]) >= 1 and sum(want["lengths"]) >= 10
