"""CPU checks of the vectorised DQN training pieces.

* The oracle's minibatch sampler (se_replay_sample's contract) is a keyed bijection
  on [0, D), so a batch holds distinct transitions like random.sample
  (agents/dqn.py:213). It skips flagged transitions, and covers the domain
  uniformly.
* dqn_loss is update()'s loss (agents/dqn.py:226-234, nn.MSELoss) when all weights
  are 1, and the MSE over the weighted rows otherwise.
* One eager update step with dqn_loss + Adam equals the reference's update code on
  the same minibatch.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
O = pytest.importorskip("oracle.oracle")


@pytest.mark.parametrize("D", [1, 2, 3, 4, 5, 31, 32, 33, 1000, 4097, 65536, 65537, 200003])
def test_feistel_is_a_bijection(D):
    key = O.philox([0xFFFFFFFF, 0xFFFFFFFF, 7, 15], [11, 0])
    p = np.array([O.feistel_perm(i, D, key) for i in range(D)])
    assert p.min() >= 0 and p.max() < D
    assert len(np.unique(p)) == D


def test_pick_distinct_and_keyed():
    size, B = 50000, 4096
    inv = np.zeros(size, np.uint8)
    a = O.replay_pick(size, B, inv, seed=5, t=0)
    b = O.replay_pick(size, B, inv, seed=5, t=1)
    c = O.replay_pick(size, B, inv, seed=6, t=0)
    assert (a >= 0).all() and len(np.unique(a)) == B
    assert (a != b).mean() > 0.99 and (a != c).mean() > 0.99
    np.testing.assert_array_equal(a, O.replay_pick(size, B, inv, seed=5, t=0))


def test_pick_is_uniform_over_the_domain():
    size, B, T = 1000, 100, 400
    inv = np.zeros(size, np.uint8)
    hits = np.zeros(size)
    for t in range(T):
        hits[O.replay_pick(size, B, inv, seed=1, t=t)] += 1
    # each index: Binomial(T, B / size) -> mean 40, sd ~6
    assert abs(hits.mean() - T * B / size) < 1e-9
    assert hits.min() > 10 and hits.max() < 75
    # chi-square over 10 bins of 100 indices
    binned = hits.reshape(10, 100).sum(1)
    chi2 = ((binned - binned.mean()) ** 2 / binned.mean()).sum()
    assert chi2 < 30


def test_pick_skips_flagged_and_reports_none():
    size, B = 1000, 200
    inv = np.zeros(size, np.uint8)
    inv[::3] = 1
    s = O.replay_pick(size, B, inv, seed=2, t=3)
    got = s[s >= 0]  # a slot is empty when its 4 positions are all flagged: p = (1/3)^4
    assert not inv[got].any() and len(np.unique(got)) == len(got) and len(got) >= 0.95 * B
    inv[:] = 1
    assert (O.replay_pick(size, B, inv, seed=2, t=3) == -1).all()
    # positions beyond size: B > size leaves slots empty
    inv[:] = 0
    s = O.replay_pick(10, 16, inv, seed=2, t=3)
    assert sorted(s[s >= 0].tolist()) == list(range(10)) and (s[10:] == -1).all()


def test_replay_memory_is_fifo():
    m = O.ReplayMemory(5, 2)
    for k in range(3):  # 9 pushes into 5 slots: slots hold pushes 5..8 and 4
        obs = np.full((3, 2), k, np.float32)
        m.push(obs, np.arange(3) + 3 * k, np.zeros(3), obs + 1, np.zeros(3), np.zeros(3))
    assert m.size == 5 and m.head == 4
    assert sorted(m.act.tolist()) == [4, 5, 6, 7, 8]


def _batch(B, width, A, seed=0, weight=None):
    from shippingenv_amd.dqn import MiniBatch

    g = torch.Generator().manual_seed(seed)
    b = MiniBatch(B, width, "cpu")
    b.obs.copy_(torch.randn(B, width, generator=g) * 10)
    b.next_obs.copy_(torch.randn(B, width, generator=g) * 10)
    b.act.copy_(torch.randint(0, A, (B,), generator=g))
    b.rew.copy_(torch.randn(B, generator=g))
    b.done.copy_((torch.rand(B, generator=g) < 0.2).float())
    b.weight.copy_(torch.ones(B) if weight is None else weight)
    return b


def _reference_update(model, target, opt, b, gamma):
    """agents/dqn.py:226-242 on the given minibatch tensors."""
    current_q = model(b.obs).gather(1, b.act.unsqueeze(1))
    with torch.no_grad():
        next_q = target(b.next_obs).max(1)[0]
        target_q = b.rew + (gamma * next_q * (1 - b.done))
    loss = torch.nn.MSELoss()(current_q.squeeze(), target_q)
    opt.zero_grad()
    loss.backward()
    opt.step()
    return loss


def test_loss_is_mse_and_masks_weight_zero_rows():
    from shippingenv_amd.dqn import dqn_loss
    from shippingenv_amd.policy import DQNNetwork

    torch.manual_seed(0)
    m, tg = DQNNetwork(26, 259), DQNNetwork(26, 259)
    b = _batch(64, 26, 259)
    q = m(b.obs).gather(1, b.act.unsqueeze(1)).squeeze(1)
    with torch.no_grad():
        tq = b.rew + 0.95 * tg(b.next_obs).max(1)[0] * (1 - b.done)
    want = torch.nn.MSELoss()(q, tq)
    got = dqn_loss(m, tg, b, 0.95)
    assert abs(float(got) - float(want)) <= 1e-6 * abs(float(want))
    w = torch.ones(64)
    w[::4] = 0
    b.weight.copy_(w)
    keep = w.bool()
    want = torch.nn.MSELoss()(q[keep], tq[keep])
    assert abs(float(dqn_loss(m, tg, b, 0.95)) - float(want)) <= 1e-6 * abs(float(want))


def test_update_step_matches_reference_update():
    from shippingenv_amd.dqn import dqn_loss
    from shippingenv_amd.policy import DQNNetwork

    torch.manual_seed(1)
    ours, ref = DQNNetwork(26, 259), DQNNetwork(26, 259)
    ref.load_state_dict(ours.state_dict())
    tg = DQNNetwork(26, 259)
    o1 = torch.optim.Adam(ours.parameters(), lr=1e-3)
    o2 = torch.optim.Adam(ref.parameters(), lr=1e-3)
    for k in range(5):
        b = _batch(32, 26, 259, seed=k)
        l1 = dqn_loss(ours, tg, b, 0.95)
        o1.zero_grad(set_to_none=False)
        l1.backward()
        o1.step()
        l2 = _reference_update(ref, tg, o2, b, 0.95)
        assert abs(float(l1) - float(l2)) <= 1e-5 * abs(float(l2))
    for p, q in zip(ours.parameters(), ref.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)
