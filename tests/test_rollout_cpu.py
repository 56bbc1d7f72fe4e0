"""The oracle's random policy and rollout loop (CPU).

sample_action (shipping/environment.py:245-263): the result's category is a
function of the state, pinned by tests/golden/sample_golden.json, which the
reference itself produced (tests/golden/make_sample_golden.py). The value is
drawn; the oracle's must lie in the same support. The rollout loop
(agents/mcts.py:211-238) is checked by its invariants; its draws follow the
production RNG contract, so GPU parity is against the oracle (test_gpu_rollout.py).
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden_water

O = pytest.importorskip("oracle.oracle")

MOVES = {(0, -1), (-1, 0), (0, 1), (1, 0)}


def fixture_world_state():
    doc = json.load(open(os.path.join(GOLDEN, "sample_golden.json")))
    ports = doc["ports"]
    world = O.OracleWorld(golden_water(), [p[0] for p in ports], [p[1] for p in ports],
                          doc["port_fuel"], doc["port_cargo"])
    recs = doc["states"]
    st = O.OracleState(len(recs))
    for i, r in enumerate(recs):
        st.x[i], st.y[i] = r["x"], r["y"]
        st.fuel[i] = r["fuel"]
        st.cargo[i] = r["cargo"]
        st.origin[i] = -1 if r["origin"] is None else r["origin"]
        st.dest[i] = -1 if r["dest"] is None else r["dest"]
    return doc, world, st


@pytest.mark.parametrize("t", [0, 1, 17])
def test_sample_action_matches_reference_categories(t):
    doc, world, st = fixture_world_state()
    ty, a, b = O.sample_actions(world, st, seed=99, t=t)
    ports = [tuple(p) for p in doc["ports"]]
    for i, r in enumerate(doc["states"]):
        out = r["out"]
        if "raise" in out:
            assert ty[i] == -1, (i, r)  # SE_SAMPLE_RAISES
            continue
        assert ty[i] == out["type"], (i, r, ty[i])
        cur = ports.index((r["x"], r["y"])) if (r["x"], r["y"]) in ports else None
        if ty[i] == 2:
            assert 0 <= a[i] < len(ports) and a[i] != cur and out["a"] != cur
        elif ty[i] == 4:
            assert 1 <= a[i] <= doc["port_cargo"][cur] and 1 <= out["a"] <= doc["port_cargo"][cur]
        else:
            assert (a[i], b[i]) in MOVES and (out["a"], out["b"]) in MOVES


def test_sample_action_values_cover_the_support():
    doc, world, st = fixture_world_state()
    moves, selects = set(), set()
    for t in range(40):
        ty, a, b = O.sample_actions(world, st, seed=5, t=t)
        moves |= {(int(x), int(y)) for x, y in zip(a[ty == 1], b[ty == 1])}
        selects |= set(a[ty == 2].tolist())
    assert moves == MOVES and selects == set(range(5))


def test_rollout_invariants():
    doc, world, st = fixture_world_state()
    n = st.n
    src = np.arange(n, dtype=np.int32)
    src[:3] = [-1, n, n + 7]  # out of range
    ret, steps, status = O.rollout(world, st, src, max_steps=60, max_attempts=480, seed=3)
    assert (status[:3] == 4).all() and (steps[:3] == 0).all() and (ret[:3] == 0).all()
    raising = np.array(["raise" in r["out"] for r in doc["states"]])
    # a state whose sample_action raises ends its rollout at the first attempt
    assert (status[3:][raising[3:]] == 2).all() and (steps[3:][raising[3:]] == 0).all()
    s3, k3 = status[3:], steps[3:]
    assert (k3 <= 60).all()
    assert (k3[s3 == 1] == 60).all()  # MAX_STEPS: exactly max_steps counted
    assert ((k3[s3 == 0] >= 1) & (k3[s3 == 0] <= 60)).all()  # DONE on a counted step
    assert (k3[s3 == 3] < 60).all()  # ATTEMPTS: the retry budget ran out first
    assert set(np.unique(s3).tolist()) >= {0, 1, 2}
    # deterministic, and independent of the other rollouts in the batch
    ret2, steps2, status2 = O.rollout(world, st, src[::-1].copy(), max_steps=60, max_attempts=480,
                                      seed=3)
    assert not np.array_equal(ret2, ret[::-1]) or n == 1  # rollout ids follow positions
    sub = O.rollout(world, st, src[10:20].copy(), max_steps=60, max_attempts=480, seed=3,
                    rollout_base=10)
    np.testing.assert_array_equal(sub[0], ret[10:20])
    np.testing.assert_array_equal(sub[1], steps[10:20])
    # the source state is not modified
    _, world2, st2 = fixture_world_state()
    for f in ("x", "y", "fuel", "cargo", "origin", "dest"):
        np.testing.assert_array_equal(getattr(st, f), getattr(st2, f))


def test_rollout_zero_budgets():
    _, world, st = fixture_world_state()
    src = np.arange(50, dtype=np.int32)
    ret, steps, status = O.rollout(world, st, src, max_steps=0, max_attempts=10, seed=1)
    # the loop condition is tested before sampling (mcts.py:225): nothing runs
    assert (status == 1).all() and (steps == 0).all() and (ret == 0).all()
    ret, steps, status = O.rollout(world, st, src, max_steps=10, max_attempts=0, seed=1)
    assert (status == 3).all() and (steps == 0).all()
