"""Batched random policy and MCTS rollouts on the GPU vs the oracle, bit for bit.

se_sample_actions (shipping/environment.py:245-263) and se_rollout
(agents/mcts.py:211-238) draw from the production RNG contract, so the checker is
the C restatement (oracle/), whose decision structure tests/test_rollout_cpu.py
pins against the reference's own sample_action (tests/golden/sample_golden.json).
"""
import numpy as np
import pytest

from test_rollout_cpu import fixture_world_state

torch = pytest.importorskip("torch")
O = pytest.importorskip("oracle.oracle")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    from shippingenv_amd import build

    build.build(verbose=False)


def VecEnv(*a, **k):
    from shippingenv_amd.vec import VecEnv as V

    return V(*a, **k)


def load_state(env, st):
    """Oracle SoA (origin/dest -1 = None) -> the device state."""
    dev = env.device
    env.x.copy_(torch.as_tensor(st.x.astype(np.uint8), device=dev))
    env.y.copy_(torch.as_tensor(st.y.astype(np.uint8), device=dev))
    env.fuel.copy_(torch.as_tensor(st.fuel, device=dev))
    env.cargo.copy_(torch.as_tensor(st.cargo, device=dev))
    env.origin.copy_(torch.as_tensor(np.where(st.origin < 0, 255, st.origin).astype(np.uint8), device=dev))
    env.dest.copy_(torch.as_tensor(np.where(st.dest < 0, 255, st.dest).astype(np.uint8), device=dev))


def oracle_state(env):
    st = O.OracleState(env.n)
    st.x[:] = env.x.cpu().numpy()
    st.y[:] = env.y.cpu().numpy()
    st.fuel[:] = env.fuel.cpu().numpy()
    st.cargo[:] = env.cargo.cpu().numpy()
    o, d = env.origin.cpu().numpy().astype(np.int32), env.dest.cpu().numpy().astype(np.int32)
    st.origin[:] = np.where(o == 255, -1, o)
    st.dest[:] = np.where(d == 255, -1, d)
    return st


def fixture_env(seed):
    doc, world, st = fixture_world_state()
    env = VecEnv(st.n, seed=seed, ports=doc["ports"], port_fuel=doc["port_fuel"],
                 port_cargo=doc["port_cargo"])
    load_state(env, st)
    return env, world, st


@pytest.mark.parametrize("t", [0, 3, 1000])
def test_sample_actions_vs_oracle_on_reference_states(t):
    env, world, st = fixture_env(seed=41)
    ty, a, b = env.sample_actions(t)
    rt, ra, rb = O.sample_actions(world, st, seed=41, t=t)
    np.testing.assert_array_equal(ty.cpu().numpy(), rt)
    np.testing.assert_array_equal(a.cpu().numpy(), ra)
    np.testing.assert_array_equal(b.cpu().numpy(), rb)
    env.close()


def test_rollouts_vs_oracle_on_reference_states():
    env, world, st = fixture_env(seed=8)
    n = env.n
    src = np.arange(n, dtype=np.int32)
    src[[5, 9]] = [-3, n]
    ret, steps, status = env.rollout(src, max_steps=100, max_attempts=800, rollout_base=1234)
    r_ret, r_steps, r_status = O.rollout(world, st, src, max_steps=100, max_attempts=800, seed=8,
                                         rollout_base=1234)
    np.testing.assert_array_equal(status.cpu().numpy(), r_status)
    np.testing.assert_array_equal(steps.cpu().numpy(), r_steps)
    np.testing.assert_array_equal(ret.cpu().numpy().view(np.uint64), r_ret.view(np.uint64))
    assert set(np.unique(r_status).tolist()) >= {0, 1, 2, 4}
    # the source envs are untouched
    after = oracle_state(env)
    for f in ("x", "y", "fuel", "cargo", "origin", "dest"):
        np.testing.assert_array_equal(getattr(after, f), getattr(st, f), err_msg=f)
    env.close()


@pytest.mark.parametrize("n,k", [(2048, 4), (1, 5), (3, 2)])
def test_rollouts_from_stepped_states_and_sampled_policy(n, k):
    """Envs driven by the batched random policy (sample -> step_typed), then K
    rollouts per env, as MCTS batches its simulations (also for one env and for three,
    the smallest batches)."""
    from shippingenv_amd.vec import random_water_ports
    from conftest import golden_water

    seed = 19
    ports = random_water_ports(golden_water(), 12, seed=4)
    env = VecEnv(n, seed=seed, ports=ports)
    env.reset()
    world = O.OracleWorld(golden_water(), env.port_x, env.port_y, env.port_fuel, env.port_cargo)
    st = oracle_state(env)
    for t in range(60):
        ty, a, b = env.sample_actions(t)
        rt, ra, rb = O.sample_actions(world, st, seed=seed, t=t)
        np.testing.assert_array_equal(ty.cpu().numpy(), rt)
        np.testing.assert_array_equal(a.cpu().numpy(), ra)
        keep = rt >= 0  # the device reports a raising sample as BAD_CATEGORY; skip those in both
        rt = np.where(keep, rt, 0)
        env.step_typed(torch.as_tensor(rt, device=env.device), a, b)
        O.step(world, st, act_type=rt, act_a=ra, act_b=rb, seed=seed, t=t)
        np.testing.assert_array_equal(env.reward.cpu().numpy(), st.reward.astype(np.float32))
    src = np.repeat(np.arange(n, dtype=np.int32), k)
    ret, steps, status = env.rollout(src, max_steps=100, rollout_base=7 * n)
    r = O.rollout(world, oracle_state(env), src, max_steps=100, max_attempts=800, seed=seed,
                  rollout_base=7 * n)
    np.testing.assert_array_equal(ret.cpu().numpy().view(np.uint64), r[0].view(np.uint64))
    np.testing.assert_array_equal(steps.cpu().numpy(), r[1])
    np.testing.assert_array_equal(status.cpu().numpy(), r[2])
    # rollouts of one env differ (independent streams) but share the start state
    if n >= 64:
        rr = ret.cpu().numpy().reshape(n, k)
        assert (rr.std(axis=1) > 0).mean() > 0.5
    env.close()
