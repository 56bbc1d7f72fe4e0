"""The N>1 path on CPU: two gloo ranks each step their shard of global env ids
(the oracle stands in for the kernel here) and all-reduce the episode stats;
the result equals one process stepping all ids. Ports and seeds as config 4."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT

N, T, SEED = 4096, 300, 77


def _world_setup(water):
    from shippingenv_amd.vec import draw_port_stocks, random_water_ports

    ports = random_water_ports(water, 64, seed=3)
    pf, pc = draw_port_stocks(64, SEED)
    return ports, pf, pc


def _run_shard(first, count, water):
    import sys

    sys.path.insert(0, ROOT)
    from oracle import oracle as O

    ports, pf, pc = _world_setup(water)
    world = O.OracleWorld(water, [p[0] for p in ports], [p[1] for p in ports], pf, pc)
    st = O.OracleState(count)
    O.reset(world, st, seed=SEED, env_id_base=first, epoch=0)
    stats = np.zeros(3)
    for t in range(T):
        acts = O.gen_actions(count, 64, SEED, first, t)
        O.step_autoreset(world, st, acts, seed=SEED, env_id_base=first, t=t, stats=stats)
    return stats, st


def _worker(rank, world_size, port, water, out):
    import sys

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world_size), LOCAL_RANK=str(rank))
    from shippingenv_amd import dist as D

    r, w, _, dev = D.init_from_env(backend="gloo")
    assert (r, w) == (rank, world_size)
    first, count = D.shard_bounds(N, w, r)
    stats, st = _run_shard(first, count, water)
    t = torch.tensor(stats, dtype=torch.float64)
    D.reduce_episode_stats(t)
    out[rank] = (t.tolist(), first, st.x.tolist()[:64], st.fuel.tolist()[:64])
    torch.distributed.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_gloo_matches_single_process(water):
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(2, _free_port(), water, out), nprocs=2, join=True,
                       start_method="spawn")
    whole, st_all = _run_shard(0, N, water)
    for rank in range(2):
        red, first, x, fuel = out[rank]
        assert red[1] == whole[1] and red[2] == whole[2]  # episodes, lengths: exact
        np.testing.assert_allclose(red[0], whole[0], rtol=1e-12)  # f64 sum order differs
        # the shard's envs are the same global ids as in the single-process run
        np.testing.assert_array_equal(x, st_all.x[first:first + 64])
        np.testing.assert_array_equal(np.asarray(fuel).view(np.int64),
                                      st_all.fuel[first:first + 64].view(np.int64))
    assert whole[1] > 0


def test_shard_bounds_rules():
    from shippingenv_amd.dist import shard_bounds

    assert shard_bounds(1 << 20, 8, 3) == (3 << 17, 1 << 17)
    with pytest.raises(ValueError):
        shard_bounds(4096 + 4, 2, 0)


def test_sharded_env_attribute_lookup_without_env():
    """A ShardedVecEnv whose __init__ failed before self.env was set answers attribute
    lookups with AttributeError, not a RecursionError through __getattr__."""
    from shippingenv_amd.dist import ShardedVecEnv

    s = object.__new__(ShardedVecEnv)
    assert not hasattr(s, "env") and not hasattr(s, "n")
    repr(s)


# ------------------------------------------------- data-parallel DQN gradient exchange
def _grad_sums(seed, rows, lay):
    """float64 sums of sum w (q - y)^2 gradients of a fixed DQNNetwork over a seeded
    minibatch of `rows` rows, laid out as shippingenv_amd.dqn.grad_layout (P = 5)."""
    import sys

    sys.path.insert(0, ROOT)
    from shippingenv_amd.policy import DQNNetwork

    torch.manual_seed(0)
    m, tg = DQNNetwork(26, 259).double(), DQNNetwork(26, 259).double()
    g = torch.Generator().manual_seed(seed)
    obs = torch.rand((rows, 26), generator=g, dtype=torch.float64) * 100
    nxt = torch.rand((rows, 26), generator=g, dtype=torch.float64) * 100
    act = torch.randint(0, 259, (rows,), generator=g)
    rew = torch.randn(rows, generator=g, dtype=torch.float64)
    done = (torch.rand(rows, generator=g) < 0.1).double()
    w = (torch.rand(rows, generator=g) < 0.9).double()  # some rows invalid (weight 0)
    q = m(obs).gather(1, act.unsqueeze(1)).squeeze(1)
    with torch.no_grad():
        y = rew + 0.95 * tg(nxt).max(1)[0] * (1 - done)
    ls = (w * (q - y) ** 2).sum()
    ls.backward()
    v = torch.zeros(lay["size"], dtype=torch.float64)
    v[lay["w1d"]:lay["w1d"] + 768] = m.fc1.weight.grad[:, :6].reshape(-1)
    v[lay["b1"]:lay["b1"] + 128] = m.fc1.bias.grad
    v[lay["w2"]:lay["w2"] + 128 * 128] = m.fc2.weight.grad.reshape(-1)
    v[lay["b2"]:lay["b2"] + 128] = m.fc2.bias.grad
    v[lay["w3"]:lay["w3"] + 259 * 128] = m.fc3.weight.grad.reshape(-1)
    v[lay["b3"]:lay["b3"] + 259] = m.fc3.bias.grad
    v[lay["lw"]], v[lay["lw"] + 1] = ls.detach(), w.sum()
    return v


def _grad_worker(rank, world_size, port, out):
    import sys

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world_size), LOCAL_RANK=str(rank))
    from shippingenv_amd import dist as D
    from shippingenv_amd.dqn import grad_layout

    D.init_from_env(backend="gloo")
    lay = grad_layout(259, 26)
    v = _grad_sums(1000 + rank, 96, lay).float()
    D.allreduce_gradient(v)
    with pytest.raises(ValueError):
        D.allreduce_gradient(v.double())
    out[rank] = v.tolist()
    torch.distributed.destroy_process_group()


def test_two_rank_gradient_exchange_is_the_union_batch():
    """The data-parallel exchange (dist.allreduce_gradient over gloo, 2 ranks): each rank's
    vector of undivided gradient sums, summed, is the union minibatch's vector, so
    grad / sum w is the union's nn.MSELoss gradient even when the ranks hold different
    numbers of valid (weight-1) rows."""
    from shippingenv_amd.dqn import grad_layout

    lay = grad_layout(259, 26)
    assert lay["size"] == 896 + 128 * 128 + 128 + 288 * 128 + 288 + 2
    ctx = mp.get_context("spawn")
    out = ctx.Manager().dict()
    mp.start_processes(_grad_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    a, b = (torch.tensor(out[r], dtype=torch.float64) for r in range(2))
    assert torch.equal(a, b)  # every rank holds the same sums
    whole = _grad_sums(1000, 96, lay) + _grad_sums(1001, 96, lay)
    scale = whole.abs().max()
    assert float((a - whole).abs().max()) <= 1e-6 * float(scale)  # f32 on the wire
