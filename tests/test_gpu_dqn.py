"""The device replay ring, the minibatch sampler and the vectorised DQN update
(agents/dqn.py:117-123 remember, :206-245 update) vs the oracle and
the reference's update code.

Bars:
* Ring plus sampler: the minibatch equals, bit for bit, the oracle's.
  * The oracle is a FIFO of full preprocess_state rows (O.ReplayMemory, as the
    reference's deque holds them).
  * Its indices come from the sampler contract (O.replay_pick).
  * The actions include invalid ones, so flagged transitions and episode cuts occur.
* The cut mask is err != 0 | ep_len >= max_steps, exactly.
* Update: on the minibatch the agent drew, one step of the reference's update()
  (nn.MSELoss, Adam) in float64 gives the loss (rtol 1e-4) and, per element, the
  weights and Adam moments within what f32 rounding of the gradient can move them
  (_Ref64).
* Graph replay and eager updates give the same trajectory: actions, states, losses,
  weights; so do the fused launches and the separate ones.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
O = pytest.importorskip("oracle.oracle")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    from shippingenv_amd import build

    build.build(verbose=False)


_OPEN = []


@pytest.fixture(autouse=True)
def _close_after():
    yield
    while _OPEN:  # agents / buffers before their env, also when the test failed
        _OPEN.pop().close()


def make_env(n, seed, ports=None):
    from shippingenv_amd.vec import VecEnv

    env = VecEnv(n, seed=seed, ports=ports, auto_reset=True)
    _OPEN.append(env)
    env.reset()
    return env


def rows(world, env):
    """preprocess_state rows of the env's current state, from the oracle."""
    torch.cuda.synchronize()
    st = O.OracleState(env.n)
    st.x[:] = env.x.cpu().numpy()
    st.y[:] = env.y.cpu().numpy()
    st.fuel[:] = env.fuel.cpu().numpy()
    for f in ("origin", "dest"):
        v = getattr(env, f).cpu().numpy().astype(np.int32)
        getattr(st, f)[:] = np.where(v == 255, -1, v)
    return O.observe(world, st)


def test_max_steps_needs_auto_reset():
    """se_replay_end refuses max_steps > 0 on an env without auto-reset, whose
    episode-start stamps only reset writes (a length cut there would count from the last
    reset, not from the episode's start); max_steps = 0 still records."""
    from shippingenv_amd._native import ShipEnvError
    from shippingenv_amd.dqn import ReplayBuffer
    from shippingenv_amd.vec import VecEnv

    env = VecEnv(256, seed=1)
    _OPEN.append(env)
    env.reset()
    rb = ReplayBuffer(env, 1024)
    _OPEN.append(rb)
    cut = torch.zeros(256, dtype=torch.uint8, device=env.device)
    a = env.gen_actions(0)
    rb.begin(a)
    env.step(a)
    with pytest.raises(ShipEnvError, match="max_steps"):
        rb.end(cut, 4)
    rb.end(cut, 0)
    assert rb.size == 256


@pytest.mark.parametrize("n,cap,ports64", [(1000, 2500, False), (4099, 20000, True)])
def test_replay_ring_and_minibatch_vs_oracle(n, cap, ports64):
    from conftest import golden_water
    from shippingenv_amd.dqn import MiniBatch, ReplayBuffer
    from shippingenv_amd.vec import random_water_ports

    ports = random_water_ports(golden_water(), 64, seed=3) if ports64 else None
    env = make_env(n, seed=7, ports=ports)
    world = O.OracleWorld(env.water, env.port_x, env.port_y, env.port_fuel, env.port_cargo)
    rb = ReplayBuffer(env, cap)
    _OPEN.append(rb)
    mem = O.ReplayMemory(cap, env.obs_size)
    cut = torch.zeros(n, dtype=torch.uint8, device=env.device)
    max_steps = 4
    flagged = cuts = 0
    for t in range(7):
        a = env.gen_actions(t)
        s_rows = rows(world, env)
        rb.begin(a)
        env.step(a)
        rb.end(cut, max_steps)
        torch.cuda.synchronize()
        r, d = env.reward.cpu().numpy(), env.done.cpu().numpy()
        e, epl = env.err.cpu().numpy(), env.ep_len.cpu().numpy()
        mem.push(s_rows, a.cpu().numpy(), r, rows(world, env), d, e != 0)
        want_cut = ((e != 0) | (epl >= max_steps)).astype(np.uint8)
        np.testing.assert_array_equal(cut.cpu().numpy(), want_cut, err_msg=f"cut at step {t}")
        flagged += int((e != 0).sum())
        cuts += int(want_cut.sum())
        env.reset(cut)
    assert flagged > 0 and cuts > flagged  # both kinds of episode break occurred
    assert rb.size == mem.size == min(7 * n, cap)
    names = ("obs", "next_obs", "act", "rew", "done", "weight")
    for B, t in [(700, 0), (cap // 2, 3), (cap + 100, 9)]:
        out = MiniBatch(B, env.obs_size, env.device)
        rb.sample(out, t=t)
        torch.cuda.synchronize()
        want = mem.sample(B, seed=env.seed, t=t)
        for name, w in zip(names, want):
            np.testing.assert_array_equal(getattr(out, name).cpu().numpy(), w, err_msg=f"{name} B={B} t={t}")
        if B <= cap // 2:  # an empty slot needs all of its (<= 4) positions flagged
            assert out.weight.mean().item() > 0.95
        # the device counter keys the same draw as the host t
        ctr = torch.full((1,), t, dtype=torch.int32, device=env.device)
        out2 = MiniBatch(B, env.obs_size, env.device)
        rb.sample(out2, t=12345, t_dev=ctr)
        torch.cuda.synchronize()
        for name in names:
            assert torch.equal(getattr(out, name), getattr(out2, name)), name


_BETA1, _BETA2, _ADAM_EPS = 0.9, 0.999, 1e-8  # torch.optim.Adam defaults (agents/dqn.py:106)
_GRAD_NOISE = 1e-3  # allowed gradient error floor, as a share of the tensor's rms gradient
_ORDERS, _SPREAD_MARGIN = 8, 10.0  # f32 gradients over batch orders; margin on their spread


def _grad32_spread(model, target, b, gamma, g64):
    """Per element, the largest distance of an f32 gradient of the reference's loss from the
    float64 one over _ORDERS orders of the minibatch (the mean is order-free; its f32 sums
    are not): how much f32 summation order alone moves that element."""
    import copy

    gen = torch.Generator(device="cpu").manual_seed(1234)
    spread = [torch.zeros_like(g) for g in g64]
    for _ in range(_ORDERS):
        perm = torch.randperm(b.obs.shape[0], generator=gen).to(b.obs.device)
        m = copy.deepcopy(model).float()
        q = m(b.obs[perm]).gather(1, b.act[perm].unsqueeze(1))
        with torch.no_grad():
            next_q = target.float()(b.next_obs[perm]).max(1)[0]
            target_q = b.rew[perm] + (gamma * next_q * (1 - b.done[perm]))
        torch.nn.MSELoss()(q.squeeze(), target_q).backward()
        for s, p, g in zip(spread, m.parameters(), g64):
            torch.maximum(s, (p.grad.double() - g).abs(), out=s)
    return spread


class _Ref64:
    """One step of the reference's update() (agents/dqn.py:226-242: nn.MSELoss, then
    torch.optim.Adam) in float64, from given parameters, Adam moments and steps taken, on
    the minibatch the agent drew. float64 takes the reference side's own summation order
    out of the comparison (torch's f32 backward does not sum in a fixed order on ROCm).

    The f32 path under test sums the gradient in some order of its own. Its error is
    bounded per element by Δ = max(_GRAD_NOISE x rms(g) of the tensor, _SPREAD_MARGIN x
    the element's spread over _ORDERS f32 batch orders): elements whose sums cancel
    (W1's fuel and port columns hold values up to 200) move with the order, the rest
    by ~1e-5 of the rms, and a wrong gradient, wrong by O(rms) (one sample of 256
    dropped is caught), is far outside either. Adam turns Δ into a per-element
    parameter bound: the largest move of m̂/(√v̂+ε) over gradients in [g − Δ, g + Δ].
    Elements whose gradient cancels to ≈ 0 get up to 2 lr (the sign of a near-zero
    gradient is decided by rounding); all others are held to f32 rounding."""

    def __init__(self, model, target, b, gamma, lr, steps, exp_avg=None, exp_avg_sq=None):
        import copy

        m = copy.deepcopy(model).double()
        tg = copy.deepcopy(target).double()
        self.lr, self.t = lr, steps + 1
        q = m(b.obs.double()).gather(1, b.act.unsqueeze(1))
        with torch.no_grad():
            next_q = tg(b.next_obs.double()).max(1)[0]
            target_q = b.rew.double() + (gamma * next_q * (1 - b.done.double()))
        self.loss = torch.nn.MSELoss()(q.squeeze(), target_q)
        m.zero_grad()
        self.loss.backward()
        self.g = [p.grad.detach().clone() for p in m.parameters()]
        self.p0 = [p.detach().clone() for p in m.parameters()]
        z = [torch.zeros_like(p) for p in self.p0]
        self.m0 = [t.double() for t in exp_avg] if steps else z
        self.v0 = [t.double() for t in exp_avg_sq] if steps else z
        opt = torch.optim.Adam(m.parameters(), lr=lr)
        if steps:
            for p, m0, v0 in zip(m.parameters(), self.m0, self.v0):
                opt.state[p] = {"step": torch.tensor(float(steps)), "exp_avg": m0.clone(), "exp_avg_sq": v0.clone()}
        opt.step()
        self.p = [p.detach() for p in m.parameters()]
        self.m = [opt.state[p]["exp_avg"] for p in m.parameters()]
        self.v = [opt.state[p]["exp_avg_sq"] for p in m.parameters()]
        spread = _grad32_spread(model, target, b, gamma, self.g)
        self.delta = [torch.clamp(_SPREAD_MARGIN * sp, min=float(_GRAD_NOISE * g.pow(2).mean().sqrt()))
                      for g, sp in zip(self.g, spread)]

    def _direction(self, i, g):
        m = _BETA1 * self.m0[i] + (1 - _BETA1) * g
        v = _BETA2 * self.v0[i] + (1 - _BETA2) * g * g
        mh, vh = m / (1 - _BETA1 ** self.t), v / (1 - _BETA2 ** self.t)
        return mh / (vh.sqrt() + _ADAM_EPS)

    def param_bound(self, i):
        r = self._direction(i, self.g[i])
        dev = torch.zeros_like(r)
        for s in torch.linspace(-1.0, 1.0, 9).tolist():
            dev = torch.maximum(dev, (self._direction(i, self.g[i] + s * self.delta[i]) - r).abs())
        return self.lr * torch.clamp(1.5 * dev, max=2.0) + 1e-6 * self.p[i].abs() + 1e-5 * self.lr

    def check(self, loss, params, exp_avg=None, exp_avg_sq=None, rtol=1e-4, what=""):
        assert abs(loss.item() - self.loss.item()) <= rtol * abs(self.loss.item()), (what, loss.item(), self.loss.item())
        names = ("w1", "b1", "w2", "b2", "w3", "b3")
        for i, (name, got) in enumerate(zip(names, params)):
            d = (got.detach().double() - self.p[i]).abs()
            bound = self.param_bound(i)
            worst = int(torch.argmax(d - bound))
            assert bool((d <= bound).all()), (what, name, "param", d.flatten()[worst].item(), bound.flatten()[worst].item())
            assert d.max().item() <= 2.0 * self.lr + 1e-6, (what, name)
        if exp_avg is None:
            return
        for i, (name, m, v) in enumerate(zip(names, exp_avg, exp_avg_sq)):
            dm = (m.double() - self.m[i]).abs()
            assert bool((dm <= (1 - _BETA1) * self.delta[i] + 1e-6 * self.m[i].abs() + 1e-30).all()), (what, name, "exp_avg")
            g = self.g[i].abs()
            dv = (v.double() - self.v[i]).abs()
            vb = (1 - _BETA2) * (2 * g * self.delta[i] + self.delta[i] ** 2) + 1e-5 * self.v[i] + 1e-30
            assert bool((dv <= vb).all()), (what, name, "exp_avg_sq")


@pytest.mark.parametrize("n,ports64,batch", [(2048, False, 256), (4099, True, 300), (4, False, 3), (64, False, 33),
                                             (16384, True, 9000)])
def test_fused_update_matches_reference_update(n, ports64, batch):
    """Per update k: from our parameters and Adam moments before it, the reference's update
    (agents/dqn.py:226-242: nn.MSELoss, torch.optim.Adam) in float64 on the minibatch the
    agent drew gives our loss (rtol 1e-4), parameters and moments within the per-element
    bounds of _Ref64. Batch 9000: 282 tiles, past the bench's 8192, so T2's sums loop over
    more than one 256-tile chunk (the action -> slot table, the W1 / W2 partials)."""
    import copy

    from conftest import golden_water
    from shippingenv_amd.dqn import VecDQNAgent
    from shippingenv_amd.vec import random_water_ports

    ports = random_water_ports(golden_water(), 64, seed=3) if ports64 else None
    env = make_env(n, seed=3, ports=ports)
    agent = VecDQNAgent(env, graph=False, batch_size=batch, epsilon=0.5, target_update_every=2)
    _OPEN.append(agent)
    tr = agent.trainer
    for k in range(5):
        before = copy.deepcopy(agent.model)
        target = copy.deepcopy(agent.target_model)
        m0 = [t.clone() for t in tr.exp_avg]
        v0 = [t.clone() for t in tr.exp_avg_sq]
        loss = agent.step()
        agent.memory.sample(agent.batch, t=k)  # the minibatch the fused update drew (key k)
        assert loss is not None and agent.batch.weight.min().item() == 1.0
        ref = _Ref64(before, target, agent.batch, agent.gamma, agent.learning_rate, k, m0, v0)
        ref.check(loss, list(agent.model.parameters()), tr.exp_avg, tr.exp_avg_sq, what=f"fused step {k}")
    assert int(agent._ctr[0].item()) == 5


def test_torch_update_matches_reference_update():
    """The torch path (fused=False: autograd + capturable Adam) against the same float64
    reference update, step by step from its own parameters and moments."""
    import copy

    from shippingenv_amd.dqn import VecDQNAgent

    env = make_env(2048, seed=3)
    agent = VecDQNAgent(env, graph=False, fused=False, batch_size=256, epsilon=0.5, target_update_every=0)
    _OPEN.append(agent)
    params = list(agent.model.parameters())
    for k in range(4):
        before = copy.deepcopy(agent.model)
        target = copy.deepcopy(agent.target_model)
        st = [agent.optimizer.state.get(p, {}) for p in params]
        m0 = [s["exp_avg"].clone() for s in st] if k else None
        v0 = [s["exp_avg_sq"].clone() for s in st] if k else None
        loss = agent.step()
        assert loss is not None
        assert agent.batch.weight.min().item() == 1.0
        ref = _Ref64(before, target, agent.batch, agent.gamma, agent.learning_rate, k, m0, v0)
        st = [agent.optimizer.state[p] for p in params]
        ref.check(loss, params, [s["exp_avg"] for s in st], [s["exp_avg_sq"] for s in st], rtol=1e-5,
                  what=f"torch step {k}")
    assert agent.epsilon == pytest.approx(0.5 * 0.995 ** 4)


def test_graph_replay_matches_eager():
    from shippingenv_amd.dqn import VecDQNAgent

    agents, envs = [], []
    for graph in (False, True):
        env = make_env(4096, seed=11)
        torch.manual_seed(0)
        agent = VecDQNAgent(env, graph=graph, graph_warmup=2, batch_size=512, epsilon=0.3,
                            target_update_every=3, max_steps=6)
        _OPEN.append(agent)
        agents.append(agent)
        envs.append(env)
    for k in range(9):
        la, lb = (a.step() for a in agents)
        assert la.item() == lb.item(), k
        assert torch.equal(agents[0].policy.actions, agents[1].policy.actions), k
        for f in ("x", "y", "fuel", "cargo", "origin", "dest", "ep_len"):
            assert torch.equal(getattr(envs[0], f), getattr(envs[1], f)), (k, f)
    assert agents[1]._graph is not None
    for p, q in zip(agents[0].model.parameters(), agents[1].model.parameters()):
        assert torch.equal(p, q)
    qs, acts = [], []
    for a in agents:
        q = torch.full((a.env.n, a.env.action_space_size), float("nan"), device=a.env.device)
        acts.append(a.policy.act(0.0, 0, q_out=q).clone())
        qs.append(q)
        acts.append(a.policy.act(0.0, 0).clone())  # the compact image
    assert torch.equal(qs[0], qs[1])
    assert torch.equal(acts[0], acts[2]) and torch.equal(acts[1], acts[3]) and torch.equal(acts[0], acts[1])


def test_vec_dqn_fits_frozen_targets_and_greedy_beats_random():
    """VERDICT r05 item 5 (agents/dqn.py:206-245, :247-347).
    (a) The fused update is a working optimiser: with the target network frozen
    (target_update_every = 0) and the replay ring no longer stepped, Q is regressed onto fixed
    targets, and the TD loss of a fixed minibatch of the ring falls to under half its start.
    (b) From reset, over 100 steps, the greedy policy of the trained network returns more per
    env than the epsilon = 1 policy (the reference's random.choice over the valid actions) on
    the same envs. (b) needs no navigation: a ship that stays in port taking cargo or fuel
    earns +0.05 a step (environment.py:341-357), the only reward a ship can collect without
    moving, where random play burns fuel and hits ground. What the reference's hyperparameters
    learn at sea is tools/dqn_learning.py's record (profiles/r06/dqn_learning/)."""
    from shippingenv_amd.dqn import MiniBatch, VecDQNAgent, dqn_loss
    from shippingenv_amd.policy import QPolicy
    from shippingenv_amd.vec import VecEnv

    n = 4096
    env = make_env(n, seed=5)
    agent = VecDQNAgent(env, batch_size=256, memory_size=4 * n, target_update_every=0, updates_per_step=0)
    _OPEN.append(agent)
    for _ in range(4):  # the ring fills (no updates: updates_per_step = 0)
        agent.step()
    fixed = MiniBatch(256, env.obs_size, env.device)
    agent.memory.sample(fixed, t=777)
    with torch.no_grad():
        loss0 = float(dqn_loss(agent.model, agent.target_model, fixed, agent.gamma))
    for _ in range(300):
        agent.update()
    with torch.no_grad():
        loss1 = float(dqn_loss(agent.model, agent.target_model, fixed, agent.gamma))
    assert np.isfinite(loss1) and loss1 < 0.5 * loss0, (loss0, loss1)

    def horizon_return(eps):
        ev = VecEnv(n, seed=6, auto_reset=True)
        _OPEN.append(ev)
        ev.reset()
        pol = QPolicy(ev, agent.model)
        _OPEN.append(pol)
        total = torch.zeros(n, dtype=torch.float64, device=ev.device)
        for t in range(100):
            ev.step(pol.act(eps, 1000 + t))
            total += ev.reward.double()
        return float(total.mean())

    greedy, rnd = horizon_return(0.0), horizon_return(1.0)
    assert greedy > rnd, (greedy, rnd)


def test_training_loop_bookkeeping():
    from shippingenv_amd.dqn import VecDQNAgent

    env = make_env(4096, seed=1)
    agent = VecDQNAgent(env, batch_size=512, memory_size=30000, max_steps=5, target_update_every=5)
    _OPEN.append(agent)
    for k in range(12):
        loss = agent.step()
        torch.cuda.synchronize()
        assert int(env.err.abs().max()) == 0  # raised steps were cut and restarted
        assert int(env.ep_len.max()) < 5       # max_steps cuts
    assert np.isfinite(loss.item())
    assert agent.updates == 12 and agent.memory.size == 30000
    assert agent.epsilon == pytest.approx(0.995 ** 12)
    assert int(agent._ctr[0].item()) == 12
    # the policy acts with the trained weights: greedy actions = argmax of the new Q
    q = torch.empty((env.n, env.action_space_size), dtype=torch.float32, device=env.device)
    agent.policy.act(0.0, 99, q_out=q)
    with torch.no_grad():
        q32 = agent.model(env.observe())
    assert float((q - q32).abs().max()) <= 0.03 * float(q32.abs().max())


@pytest.mark.parametrize("precision", ["bf16", "f32"])
def test_fused_launches_equal_the_unfused_loop(precision):
    """The training loop's fused launches (se_policy_record / se_policy_record_f32 = policy
    + remember(s, a), in the agent's precision;
    se_replay_end_reset = remember(r, s') + reset of the cut episodes; se_qtrain_step_policy
    = the update + the policy's repack + the counter's advance) give, bit for bit, what the
    separate launches give: actions, env state, losses, the update counter, the weights,
    and the Q rows of both policy images (the compact one through the greedy actions, the
    full one through q_out)."""
    from shippingenv_amd.dqn import VecDQNAgent

    class Unfused(VecDQNAgent):
        def _update_body(self):
            self.memory.sample(self.batch, t_dev=self._ctr)
            self.trainer.step(self.batch, self.gamma, self._ctr, self._loss)
            self._ctr.add_(1)
            self.policy.set_weights()

        def step(self):
            env = self.env
            a = self.choose_actions()
            self.memory.begin(a)
            env.step(a)
            self.memory.end(self.cut, self.max_steps)
            env.reset(self.cut)
            loss = None
            for _ in range(self.updates_per_step):
                loss = self.update()
            self.t += 1
            return loss

    agents, envs = [], []
    for cls in (VecDQNAgent, Unfused):
        env = make_env(4096 + 4, seed=21)
        torch.manual_seed(0)
        agent = cls(env, graph=False, batch_size=512, epsilon=0.4, target_update_every=3, max_steps=7,
                    precision=precision)
        _OPEN.append(agent)
        agents.append(agent)
        envs.append(env)
    for k in range(12):
        la, lb = (a.step() for a in agents)
        assert (la is None) == (lb is None), k
        if la is not None:
            assert la.item() == lb.item(), k
        assert torch.equal(agents[0].policy.actions, agents[1].policy.actions), k
        assert torch.equal(agents[0].cut, agents[1].cut), k
        for f in ("x", "y", "fuel", "cargo", "origin", "dest", "ep_len", "ep_return", "done", "err"):
            assert torch.equal(getattr(envs[0], f), getattr(envs[1], f)), (k, f)
        assert int(agents[0]._ctr[0].item()) == int(agents[1]._ctr[0].item()), k
    assert agents[0].memory.size == agents[1].memory.size
    assert int(agents[0]._ctr[0].item()) > 0 and int(agents[0].cut.sum()) >= 0
    for p, q in zip(agents[0].model.parameters(), agents[1].model.parameters()):
        assert torch.equal(p, q)
    qs, acts = [], []
    for a in agents:
        q = torch.full((a.env.n, a.env.action_space_size), float("nan"), device=a.env.device)
        acts.append(a.policy.act(0.0, 0, q_out=q).clone())
        qs.append(q)
        acts.append(a.policy.act(0.0, 0).clone())  # the compact image
    assert torch.equal(qs[0], qs[1])
    assert torch.equal(acts[0], acts[2]) and torch.equal(acts[1], acts[3]) and torch.equal(acts[0], acts[1])


@pytest.mark.parametrize("n,cap", [(4096, 20000), (4096, 10000), (4100, 10002), (4098, 20000)])
def test_step_record_equals_step_then_end_reset(n, cap):
    """se_step_record (one launch: the step kernel writes the ring's record and restarts the
    cut envs) against se_step + se_replay_end_reset, bit for bit: env state, cut mask, episode
    statistics and the ring, read through minibatches of every stored transition. The first
    two cases take the one-launch path (the second wraps the ring); n or the capacity not a
    multiple of 4 take the two-launch path inside se_step_record."""
    from shippingenv_amd.dqn import MiniBatch, ReplayBuffer

    envs, rbs, cuts = [], [], []
    for _ in range(2):
        env = make_env(n, seed=13)
        rb = ReplayBuffer(env, cap)
        _OPEN.append(rb)
        envs.append(env)
        rbs.append(rb)
        cuts.append(torch.zeros(n, dtype=torch.uint8, device=env.device))
    max_steps = 4
    n_cut = 0
    for t in range(9):
        a = envs[0].gen_actions(t)
        rbs[0].begin(a)
        rbs[0].step_end(a, cuts[0], max_steps)
        rbs[1].begin(a)
        envs[1].step(a)
        rbs[1].end(cuts[1], max_steps, reset=True)
        torch.cuda.synchronize()
        assert torch.equal(cuts[0], cuts[1]), t
        n_cut += int(cuts[0].sum())
        for f in ("x", "y", "fuel", "cargo", "origin", "dest", "ep_len", "ep_return", "done", "err", "reward"):
            assert torch.equal(getattr(envs[0], f), getattr(envs[1], f)), (t, f)
    assert n_cut > 0
    assert torch.equal(envs[0].episode_stats(), envs[1].episode_stats())
    assert rbs[0].size == rbs[1].size == min(9 * n, cap)
    B = rbs[0].size
    for t in (0, 5):
        outs = [MiniBatch(B, envs[0].obs_size, envs[0].device) for _ in range(2)]
        for rb, out in zip(rbs, outs):
            rb.sample(out, t=t)
        torch.cuda.synchronize()
        for name in ("obs", "next_obs", "act", "rew", "done", "weight"):
            assert torch.equal(getattr(outs[0], name), getattr(outs[1], name)), (t, name)


def test_step_record_refuses_without_begin():
    from shippingenv_amd import _native as N
    from shippingenv_amd.dqn import ReplayBuffer

    env = make_env(64, seed=1)
    rb = ReplayBuffer(env, 256)
    _OPEN.append(rb)
    cut = torch.zeros(64, dtype=torch.uint8, device=env.device)
    with pytest.raises(N.ShipEnvError, match="se_replay_begin"):
        rb.step_end(env.gen_actions(0), cut, 4)


def test_update_with_policy_refuses_a_foreign_qnet():
    """se_qtrain_step_policy writes the policy's images from the parameters it updates, so it
    refuses a qnet packed from other tensors (another model, or a copy)."""
    from shippingenv_amd import _native as N
    from shippingenv_amd.dqn import VecDQNAgent
    from shippingenv_amd.policy import DQNNetwork, QPolicy

    env = make_env(1024, seed=5)
    torch.manual_seed(0)
    agent = VecDQNAgent(env, graph=False, batch_size=64)
    _OPEN.append(agent)
    for _ in range(3):
        agent.step()
    other = QPolicy(env, DQNNetwork(env.obs_size, env.action_space_size))
    _OPEN.append(other)
    agent.memory.sample(agent.batch, t=7)
    before = [p.detach().clone() for p in agent.model.parameters()]
    ctr = int(agent._ctr[0].item())
    with pytest.raises(N.ShipEnvError, match="not packed from the online parameters"):
        agent.trainer.step_policy(agent.batch, agent.gamma, agent._ctr, agent._loss, other)
    torch.cuda.synchronize()
    assert int(agent._ctr[0].item()) == ctr  # refused before any launch
    for p, q in zip(agent.model.parameters(), before):
        assert torch.equal(p, q)
    agent.trainer.step_policy(agent.batch, agent.gamma, agent._ctr, agent._loss, agent.policy)
    torch.cuda.synchronize()
    assert int(agent._ctr[0].item()) == ctr + 1


@pytest.mark.parametrize("n,batch,with_policy,host_t", [(4096, 512, True, True), (4099, 300, False, False)])
def test_update_drawing_its_own_batch_equals_sampler_then_step(n, batch, with_policy, host_t):
    """se_qtrain_step_replay (the first kernel draws its minibatch rows from the ring) against
    se_replay_sample + se_qtrain_step_policy / se_qtrain_step on a twin agent: loss, weights,
    Adam moments, the counter and the policy's Q rows agree bit for bit, update after update,
    on a ring holding raised (flagged) transitions and with a partial last 32-sample tile.
    host_t: the sampler key and the ring size passed from the host instead of read on the
    device."""
    from shippingenv_amd.dqn import VecDQNAgent

    agents = []
    for _ in range(2):
        env = make_env(n, seed=17)
        torch.manual_seed(4)
        agent = VecDQNAgent(env, graph=False, batch_size=batch, epsilon=0.6, target_update_every=0)
        _OPEN.append(agent)
        for _ in range(3):
            agent.step()
        agents.append(agent)
    a, b = agents
    assert bool((a.memory.size >= batch))
    for k in range(4):
        ctr0 = int(a._ctr[0].item())
        a.trainer.step_replay(a.memory, batch, a.gamma, a._ctr, a._loss, a.policy if with_policy else None,
                              t=ctr0 if host_t else None)
        b.memory.sample(b.batch, t_dev=b._ctr)
        if with_policy:
            b.trainer.step_policy(b.batch, b.gamma, b._ctr, b._loss, b.policy)
        else:
            b.trainer.step(b.batch, b.gamma, b._ctr, b._loss)
            b._ctr.add_(1)
        torch.cuda.synchronize()
        assert a._ctr.tolist() == [ctr0 + 1, ctr0 + 1], k
        assert int(b._ctr[0].item()) == ctr0 + 1, k
        assert a._loss.item() == b._loss.item(), k
        for p, q in zip(a.model.parameters(), b.model.parameters()):
            assert torch.equal(p, q), k
        for p, q in zip(a.trainer.exp_avg + a.trainer.exp_avg_sq, b.trainer.exp_avg + b.trainer.exp_avg_sq):
            assert torch.equal(p, q), k
    if with_policy:
        qs = []
        for ag in agents:
            q = torch.full((ag.env.n, ag.env.action_space_size), float("nan"), device=ag.env.device)
            ag.policy.act(0.0, 0, q_out=q)
            qs.append(q)
        assert torch.equal(qs[0], qs[1])


def test_out_of_range_action_is_weight_zero():
    """A minibatch row whose action lies outside [0, A) (the reference's gather would
    raise) takes no part in the fused update: the same update as with that row's weight
    set to 0, bit for bit, and no read past W3."""
    from shippingenv_amd.dqn import VecDQNAgent

    agents = []
    for _ in range(2):
        env = make_env(2048, seed=9)
        torch.manual_seed(1)
        agent = VecDQNAgent(env, graph=False, batch_size=256)
        _OPEN.append(agent)
        for _ in range(4):
            agent.step()
        agents.append(agent)
    for a, b in zip(agents[0].model.parameters(), agents[1].model.parameters()):
        assert torch.equal(a, b)
    for ag in agents:
        ag.memory.sample(ag.batch, t=99)
    bad, ref = (ag.batch for ag in agents)
    bad.act[[0, 17]] = torch.tensor([agents[0].env.action_space_size, -3], device=bad.act.device)
    ref.weight[[0, 17]] = 0.0
    for ag, b in zip(agents, (bad, ref)):
        ag.trainer.step(b, ag.gamma, ag._ctr, ag._loss)
    torch.cuda.synchronize()
    assert agents[0]._loss.item() == agents[1]._loss.item()
    for a, b in zip(agents[0].model.parameters(), agents[1].model.parameters()):
        assert torch.equal(a, b)
    for a, b in zip(agents[0].trainer.exp_avg_sq, agents[1].trainer.exp_avg_sq):
        assert torch.equal(a, b)


# ---------------------------------------------------------------- data parallel (§8e x §8f row 3)
def _one_rank_dp():
    """VecDQNAgent's data-parallel path with a world of one: the exchange is the identity."""
    from shippingenv_amd.dqn import VecDQNAgent

    class OneRank(VecDQNAgent):
        def _broadcast_params(self):
            self.exchanges = 0

        def _exchange(self):
            self.exchanges += 1

    return OneRank


@pytest.mark.parametrize("n,batch", [(4096, 512), (16384, 9000)])
def test_grad_then_apply_is_the_fused_step_bit_for_bit(n, batch):
    """se_qtrain_grad + se_qtrain_apply (the update split at the all-reduce) against
    se_qtrain_step_policy, one rank: the same sums reach the same Adam step, so losses,
    weights, Adam moments, the update counter and both policy images agree bit for bit,
    eager and from the two captured graphs (batch 9000: T2's sums over two 256-tile chunks)."""
    from shippingenv_amd.dqn import VecDQNAgent

    agents, envs = [], []
    for cls in (VecDQNAgent, _one_rank_dp()):
        env = make_env(n, seed=13)
        torch.manual_seed(2)
        kw = dict(data_parallel=True) if cls is not VecDQNAgent else {}
        agent = cls(env, graph=True, graph_warmup=3, batch_size=batch, epsilon=0.4, target_update_every=4,
                    max_steps=9, **kw)
        _OPEN.append(agent)
        agents.append(agent)
        envs.append(env)
    assert agents[1].data_parallel and not agents[0].data_parallel
    for k in range(10):
        la, lb = (a.step() for a in agents)
        assert (la is None) == (lb is None), k
        if la is not None:
            assert la.item() == lb.item(), k
        assert torch.equal(agents[0].policy.actions, agents[1].policy.actions), k
        assert int(agents[0]._ctr[0].item()) == int(agents[1]._ctr[0].item()), k
    assert agents[1]._graphs is not None and agents[1].exchanges == 10
    for p, q in zip(agents[0].model.parameters(), agents[1].model.parameters()):
        assert torch.equal(p, q)
    for a, b in zip(agents[0].trainer.exp_avg + agents[0].trainer.exp_avg_sq,
                    agents[1].trainer.exp_avg + agents[1].trainer.exp_avg_sq):
        assert torch.equal(a, b)
    qs = []
    for a in agents:
        q = torch.full((a.env.n, a.env.action_space_size), float("nan"), device=a.env.device)
        a.policy.act(0.0, 0, q_out=q)
        qs.append(q)
    assert torch.equal(qs[0], qs[1])


class _Batch:
    def __init__(self, parts):
        for f in ("obs", "next_obs", "act", "rew", "done", "weight"):
            setattr(self, f, torch.cat([getattr(p, f) for p in parts]))
        self.batch = sum(p.batch for p in parts)


def _grad_sums64(model, target, b, gamma, lay):
    """float64 autograd of sum w (q - y)^2 (undivided) in se_qtrain_grad's layout."""
    import copy

    m = copy.deepcopy(model).double()
    tg = copy.deepcopy(target).double()
    q = m(b.obs.double()).gather(1, b.act.unsqueeze(1)).squeeze(1)
    with torch.no_grad():
        y = b.rew.double() + gamma * tg(b.next_obs.double()).max(1)[0] * (1 - b.done.double())
    w = b.weight.double()
    ls = (w * (q - y) ** 2).sum()
    ls.backward()
    v = torch.zeros(lay["size"], dtype=torch.float64, device=b.obs.device)
    A = m.fc3.out_features
    v[lay["w1d"]:lay["w1d"] + 768] = m.fc1.weight.grad[:, :6].reshape(-1)
    v[lay["b1"]:lay["b1"] + 128] = m.fc1.bias.grad
    v[lay["w2"]:lay["w2"] + 128 * 128] = m.fc2.weight.grad.reshape(-1)
    v[lay["b2"]:lay["b2"] + 128] = m.fc2.bias.grad
    v[lay["w3"]:lay["w3"] + A * 128] = m.fc3.weight.grad.reshape(-1)
    v[lay["b3"]:lay["b3"] + A] = m.fc3.bias.grad
    v[lay["lw"]] = ls.detach()
    v[lay["lw"] + 1] = w.sum()
    return v


def test_rank_gradients_sum_to_the_union_update():
    """Two ranks' minibatches, exchanged as se_qtrain_grad vectors: each vector equals the
    float64 autograd sums of its minibatch (5e-3 of the segment's rms), grad() changes no
    parameter, and se_qtrain_apply on their sum is the reference update (nn.MSELoss + Adam,
    _Ref64) on the union of the two minibatches."""
    import copy

    from shippingenv_amd.dqn import MiniBatch, VecDQNAgent, grad_layout

    env = make_env(4096, seed=5)
    agent = VecDQNAgent(env, graph=False, batch_size=256, epsilon=0.5, target_update_every=0)
    _OPEN.append(agent)
    for _ in range(3):
        agent.step()
    tr = agent.trainer
    lay = grad_layout(env.action_space_size, env.obs_size)
    assert tr.grad_size() == lay["size"]
    parts, grads = [], []
    for t in (77, 78):
        b = agent.memory.sample(MiniBatch(256, env.obs_size, env.device), t=t)
        g = torch.full((lay["size"],), float("nan"), dtype=torch.float32, device=env.device)
        before = [p.clone() for p in agent.model.parameters()] + [m.clone() for m in tr.exp_avg]
        tr.grad(b, agent.gamma, g)
        torch.cuda.synchronize()
        for x, y in zip(before, list(agent.model.parameters()) + tr.exp_avg):
            assert torch.equal(x, y)
        assert b.weight.min().item() == 1.0
        want = _grad_sums64(agent.model, agent.target_model, b, agent.gamma, lay)
        A = env.action_space_size
        segs = [("w1d", 768), ("b1", 128), ("w2", 128 * 128), ("b2", 128), ("w3", A * 128), ("b3", A), ("lw", 2)]
        for name, n in segs:
            got, ref = g[lay[name]:lay[name] + n].double(), want[lay[name]:lay[name] + n]
            tol = 5e-3 * ref.pow(2).mean().sqrt() + 1e-5 * ref.abs()
            assert bool(((got - ref).abs() <= tol).all()), (name, float((got - ref).abs().max()))
        parts.append(b)
        grads.append(g)
    k = int(agent._ctr[0].item())
    before = copy.deepcopy(agent.model)
    target = copy.deepcopy(agent.target_model)
    m0 = [t.clone() for t in tr.exp_avg]
    v0 = [t.clone() for t in tr.exp_avg_sq]
    tr.apply(grads[0] + grads[1], agent._ctr, agent._loss, agent.policy)
    torch.cuda.synchronize()
    ref = _Ref64(before, target, _Batch(parts), agent.gamma, agent.learning_rate, k, m0, v0)
    ref.check(agent._loss, list(agent.model.parameters()), tr.exp_avg, tr.exp_avg_sq, what="union")
    # the policy's images now hold the new weights: the same Q as a fresh packing
    from shippingenv_amd.policy import QPolicy

    fresh = QPolicy(env, agent.model)
    _OPEN.append(fresh)
    qa, qb = (torch.empty((env.n, env.action_space_size), device=env.device) for _ in range(2))
    agent.policy.act(0.0, 0, q_out=qa)
    fresh.act(0.0, 0, q_out=qb)
    assert torch.equal(qa, qb)


def _dp_worker(rank, world, port, out):
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from shippingenv_amd import dist as D
    from shippingenv_amd.dqn import DQNNetwork, VecDQNAgent

    r, w, _, dev = D.init_from_env(backend="gloo", gpu=0)  # the ranks share the one GPU
    env = D.ShardedVecEnv(2048, gpu=0, seed=9, auto_reset=True)  # the INTEGRATION.md recipe
    assert env.first == r * 2048
    env.reset()
    torch.manual_seed(100 + r)  # different initial weights: the broadcast must align them
    model = DQNNetwork(env.obs_size, env.action_space_size)
    init = torch.cat([p.detach().flatten() for p in model.parameters()]).cpu()
    agent = VecDQNAgent(env, graph=True, graph_warmup=2, batch_size=256, epsilon=0.5, target_update_every=3,
                        max_steps=8, model=model, data_parallel=True)
    assert agent.data_parallel
    losses = []
    for _ in range(7):
        loss = agent.step()
        losses.append(None if loss is None else loss.item())
    flat = torch.cat([p.detach().flatten() for p in agent.model.parameters()]).cpu()
    got = [None] * w
    dist.all_gather_object(got, (flat, losses, init))
    stats = env.global_episode_stats().cpu().tolist()
    out[rank] = (got, agent._graphs is not None, stats)
    agent.close()
    env.close()
    dist.destroy_process_group()


def test_data_parallel_ranks_stay_in_step():
    """Two ranks (gloo here, sharing this box's GPU; RCCL on a node) train on their own
    envs and rings: after rank 0's weights are broadcast, the summed gradients keep every
    rank's weights and losses identical, bit for bit, through eager and graph updates."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    mp.start_processes(_dp_worker, args=(2, port, out), nprocs=2, join=True, start_method="spawn")
    got, graphs, stats = out[0]
    assert stats == out[1][2]  # the episode statistics all-reduced over both shards
    (f0, l0, i0), (f1, l1, i1) = got
    assert graphs
    assert not torch.equal(i0, i1)        # the ranks started from different weights
    assert torch.equal(f0, f1)            # and train as one model
    assert not torch.equal(f0, i0)
    assert l0 == l1 and all(v is not None for v in l0[1:])


def _dp_mismatch_worker(rank, world, port, out, what="n"):
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from shippingenv_amd import dist as D
    from shippingenv_amd.dqn import VecDQNAgent
    from shippingenv_amd.vec import VecEnv

    r, w, _, dev = D.init_from_env(backend="gloo", gpu=0)  # the ranks share the one GPU
    if what == "n":  # different env counts
        env = VecEnv(2048 * (1 + r), seed=9, env_id_base=r * 4096, device=dev, auto_reset=True)
    else:  # the same count and port positions, different port stocks
        env = VecEnv(2048, seed=9, env_id_base=r * 2048, device=dev, auto_reset=True,
                     port_fuel=[5 + r, 6, 7, 8, 9], port_cargo=[10, 11, 12, 13, 14])
    env.reset()
    try:
        VecDQNAgent(env, graph=False, batch_size=256, data_parallel=True)
        out[rank] = "built"
    except ValueError as e:
        out[rank] = str(e)
    env.close()
    dist.destroy_process_group()


def test_data_parallel_refuses_unequal_ranks():
    """Ranks with different env counts would reach their first update at different
    iterations and leave an all-reduce waiting: construction refuses them on every rank."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = mp.get_context("spawn").Manager().dict()
    mp.start_processes(_dp_mismatch_worker, args=(2, port, out), nprocs=2, join=True, start_method="spawn")
    assert all("same env count" in out[r] for r in range(2)), dict(out)


def test_data_parallel_refuses_unequal_ports():
    """The exchanged gradient leaves out dW1's port columns (each rank rebuilds them from
    its own port block), so ranks whose ports differ would drift apart silently:
    construction refuses them on every rank."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = mp.get_context("spawn").Manager().dict()
    mp.start_processes(_dp_mismatch_worker, args=(2, port, out, "ports"), nprocs=2, join=True,
                       start_method="spawn")
    assert all("same ports" in out[r] for r in range(2)), dict(out)
