"""Full-size (N = 2^20) parity of the kernels the bench times, in the state mix it times.

bench.py's headline times `step_kernel<..., kSeq = true>` (VecEnv.step_seq) after a
1000-step pre-roll from reset; config 4 times the auto-reset kernel (64 ports) after the
same pre-roll. These tests run exactly those sequences on 2^20 envs and check sampled
slices of whole quads bit for bit against the C oracle (tests only) on the same global
ids: Philox draws are keyed by (seed, quad, step, slot), and a quad's LOSS_r / RESET_r
blocks go to its r-th firing / resetting env, so a slice of whole quads steps in the
oracle exactly as inside the full launch (shipping/environment.py:273-339, :227-243).
The slices start at random quad offsets, so they straddle wave and workgroup boundaries.
Each test also counts, in the oracle, the quad-steps whose draws used the rank >= 1
blocks (two envs of one quad losing cargo, or resetting, in the same step).
"""
import numpy as np
import pytest

from conftest import golden_water

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

FIELDS = ("x", "y", "fuel", "cargo", "origin", "dest")
N = 1 << 20
PREROLL, TIMED = 1000, 20
SLICES, SLICE = 16, 1024  # 16 slices of 256 quads: 4096 quads, 16384 envs


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from shippingenv_amd import build

    build.build(verbose=False)


def _slices(seed):
    rng = np.random.default_rng(seed)
    blocks = np.sort(rng.choice(N // SLICE - 1, SLICES - 1, replace=False))
    starts = [int(b) * SLICE + 4 * int(rng.integers(0, SLICE // 4)) for b in blocks]
    starts.append(N - SLICE)  # the grid's last workgroup
    return starts


class Sample:
    """The oracle on whole-quad slices [s, s + SLICE) of the global id range."""

    def __init__(self, O, env, starts, seed):
        self.O, self.starts, self.seed, self.P = O, starts, seed, env.P
        self.world = O.OracleWorld(env.water, env.port_x, env.port_y, env.port_fuel, env.port_cargo)
        self.sts = [O.OracleState(SLICE) for _ in starts]
        for st, s in zip(self.sts, starts):
            O.reset(self.world, st, seed=seed, env_id_base=s, epoch=0)
        self.loss_pairs = self.reset_pairs = 0

    def step(self, t, t_act, auto, stats=None, acts_dev=None):
        """One step: draws at the env's step counter t, the synthetic agent's row t_act."""
        O = self.O
        for st, s in zip(self.sts, self.starts):
            a = O.gen_actions(SLICE, self.P, self.seed, s, t_act)
            if acts_dev is not None:
                np.testing.assert_array_equal(a, acts_dev[s:s + SLICE])
            cargo0, origin0 = st.cargo.copy(), st.origin.copy()
            if auto:
                O.step_autoreset(self.world, st, a, seed=self.seed, env_id_base=s, t=t, stats=stats)
                self.reset_pairs += int(((st.done.reshape(-1, 4) != 0).sum(1) >= 2).sum())
            else:
                O.step(self.world, st, actions=a, seed=self.seed, env_id_base=s, t=t)
            # cargo fell with no arrival (origin unchanged): that env's gate fired and it lost
            # cargo, drawing a LOSS_r block; two in one quad means a LOSS_1 block was drawn
            lost = (st.cargo < cargo0) & (st.origin == origin0) & (st.done == 0)
            self.loss_pairs += int((lost.reshape(-1, 4).sum(1) >= 2).sum())

    def check(self, env, what, outputs=True, auto=False):
        torch.cuda.synchronize()
        for st, s in zip(self.sts, self.starts):
            sl = slice(s, s + SLICE)
            for f in FIELDS:
                got = getattr(env, f)[sl].cpu().numpy()
                want = getattr(st, f)
                if f == "fuel":
                    np.testing.assert_array_equal(got.view(np.int64), want.view(np.int64),
                                                  err_msg=f"{what} slice {s}: fuel bits")
                else:
                    if f in ("origin", "dest"):
                        got = np.where(got == 255, -1, got.astype(np.int32))
                    np.testing.assert_array_equal(got.astype(np.int32), want, err_msg=f"{what} slice {s}: {f}")
            if outputs:
                np.testing.assert_array_equal(env.reward[sl].cpu().numpy(), st.reward.astype(np.float32),
                                              err_msg=f"{what} slice {s}: reward")
                np.testing.assert_array_equal(env.done[sl].cpu().numpy().astype(np.int32), st.done,
                                              err_msg=f"{what} slice {s}: done")
                np.testing.assert_array_equal(env.err[sl].cpu().numpy().astype(np.int32), st.err,
                                              err_msg=f"{what} slice {s}: err")
            if auto:
                np.testing.assert_array_equal(env.ep_return[sl].cpu().numpy(), st.ep_return,
                                              err_msg=f"{what} slice {s}: ep_return")
                np.testing.assert_array_equal(env.ep_len[sl].cpu().numpy(), st.ep_len,
                                              err_msg=f"{what} slice {s}: ep_len")


def test_headline_kseq_after_preroll_vs_oracle(oracle_mod):
    """bench.py's headline leg: reset, 1000 pre-roll steps (VecEnv.step, action rows
    t = 10^6 + k), then 20 steps through VecEnv.step_seq (se_step_seq: the kSeq kernel),
    five one row at a time (every step's reward / done / err checked) and 15 in one call."""
    from shippingenv_amd.vec import VecEnv

    O, seed = oracle_mod, 2026
    env = VecEnv(N, seed=seed)
    smp = Sample(O, env, _slices(1), seed)
    env.reset()
    row = torch.empty(N, dtype=torch.int32, device=env.device)
    for k in range(PREROLL):
        env.step(env.gen_actions(1_000_000 + k, out=row))
        smp.step(k, 1_000_000 + k, False)
        if k in (0, 499):
            smp.check(env, f"pre-roll step {k}")
    smp.check(env, "after the pre-roll")
    pre_pairs = smp.loss_pairs
    acts = torch.stack([env.gen_actions(t) for t in range(TIMED)])
    for t in range(5):
        env.step_seq(acts[t:t + 1])
        smp.step(PREROLL + t, t, False, acts_dev=acts[t].cpu().numpy())
        smp.check(env, f"step_seq step {t}")
    env.step_seq(acts[5:])
    for t in range(5, TIMED):
        smp.step(PREROLL + t, t, False)
    smp.check(env, "step_seq steps 5..19")
    # in steady state about 3 % of ships carry cargo
    carrying = float((env.cargo > 0).float().mean())
    assert carrying < 0.2, carrying
    print(f"loss rank >= 1 quad-steps: pre-roll {pre_pairs}, timed {smp.loss_pairs - pre_pairs}; "
          f"carrying {carrying:.3f}")
    assert smp.loss_pairs >= 1
    env.close()


def test_config4_autoreset_after_preroll_vs_oracle(oracle_mod):
    """bench.py's config-4 leg: 64 random water ports, auto-reset, reset then 1000 pre-roll
    steps and 20 more (VecEnv.step), with ep_return / ep_len and the per-slice episode
    statistics against O.step_autoreset on the same global ids."""
    from shippingenv_amd.vec import VecEnv, random_water_ports

    O, seed = oracle_mod, 2026
    ports = random_water_ports(golden_water(), 64, seed=3)
    env = VecEnv(N, seed=seed, ports=ports, auto_reset=True)
    smp = Sample(O, env, _slices(2), seed)
    env.reset()
    stats = np.zeros(3)
    row = torch.empty(N, dtype=torch.int32, device=env.device)
    for k in range(PREROLL):
        env.step(env.gen_actions(1_000_000 + k, out=row))
        smp.step(k, 1_000_000 + k, True, stats=stats)
        if k in (0, 499):
            smp.check(env, f"pre-roll step {k}", auto=True)
    smp.check(env, "after the pre-roll", auto=True)
    pre_resets = smp.reset_pairs
    for t in range(TIMED):
        acts = env.gen_actions(t)
        env.step(acts)
        smp.step(PREROLL + t, t, True, stats=stats, acts_dev=acts.cpu().numpy() if t < 2 else None)
        smp.check(env, f"timed step {t}", auto=True)
        if t == TIMED - 1:  # the done list of the last step lists exactly the sampled dones
            ids = env.done_list()[0].cpu().numpy()
            for st, s in zip(smp.sts, smp.starts):
                inside = ids[(ids >= s) & (ids < s + SLICE)] - s
                np.testing.assert_array_equal(inside, np.nonzero(st.done)[0])
    print(f"reset rank >= 1 quad-steps: pre-roll {pre_resets}, timed {smp.reset_pairs - pre_resets}; "
          f"loss rank >= 1: {smp.loss_pairs}; episodes in the sample {stats[1]:.0f}")
    assert smp.reset_pairs >= 1 and smp.loss_pairs >= 1 and stats[1] > 1000
    env.close()
