"""ctypes binding of the C oracle (TEST INFRASTRUCTURE — see shipenv_oracle.h).

Imported only by tests/, ``__graft_entry__.smoke()`` and bench.py's
``cpu_baseline`` leg, always as the checker / the CPU baseline, never as the
thing shipped. The product path (``shippingenv_amd``) does not import this.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle_shipenv.so")

TAPE_DTYPE = np.dtype(
    [("u_fuel", "<f8"), ("u_gate", "<f8"), ("u_type", "<f8"), ("beta", "<f8"),
     ("arrive_dest", "<i4"), ("used", "<i4")]
)


class World(C.Structure):
    _fields_ = [
        ("H", C.c_int32), ("W", C.c_int32), ("P", C.c_int32),
        ("nonground", C.c_void_p), ("port_x", C.c_void_p), ("port_y", C.c_void_p),
        ("port_fuel", C.c_void_p), ("port_cargo", C.c_void_p),
    ]


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _lib():
    if not os.path.exists(LIB_PATH):
        build()
    lib = C.CDLL(LIB_PATH)
    P = C.c_void_p
    i64, i32, u32, u64 = C.c_int64, C.c_int32, C.c_uint32, C.c_uint64
    lib.orc_step_batch.argtypes = [P, i64, C.c_int, P, P, P, P, u64, i64, u32] + [P] * 9
    lib.orc_step_batch_autoreset.argtypes = [P, i64, P, u64, i64, u32] + [P] * 12
    lib.orc_reset_batch.argtypes = [P, i64, P, P, P, u64, i64, u32] + [P] * 6
    lib.orc_observe.argtypes = [P, i64] + [P] * 6
    lib.orc_valid_mask.argtypes = [P, i64] + [P] * 4
    lib.orc_philox4x32_10.argtypes = [P, P, P]
    lib.orc_gen_actions.argtypes = [i64, i32, u64, i64, u32, P]
    lib.orc_decode_agent.argtypes = [i32, i64, P, P, P, P, P]
    lib.orc_sample_actions.argtypes = [P, i64] + [P] * 6 + [u64, i64, u32, P, P, P]
    lib.orc_feistel_perm.argtypes = [u32, u32, P]
    lib.orc_feistel_perm.restype = u32
    lib.orc_replay_pick.argtypes = [i64, i64, P, u64, u32, P]
    lib.orc_rollout.argtypes = [P, i64] + [P] * 6 + [i64, P, i32, i32, u64, i64, P, P, P]
    return lib


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        _LIB = _lib()
    return _LIB


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class OracleWorld:
    """Static map + ports, the data add_port/_initialize_map leave behind."""

    def __init__(self, water, port_x, port_y, port_fuel, port_cargo):
        water = np.ascontiguousarray(water, np.uint8)
        self.H, self.W = water.shape
        ng = water.copy()
        px = np.ascontiguousarray(port_x, np.int32)
        py = np.ascontiguousarray(port_y, np.int32)
        ng[px, py] = 1  # add_port stamps Entity.PORT (shipping/environment.py:65)
        self.nonground = np.ascontiguousarray(ng, np.uint8)
        self.px, self.py = px, py
        self.pf = np.ascontiguousarray(port_fuel, np.int32)
        self.pc = np.ascontiguousarray(port_cargo, np.int32)
        self.P = len(px)
        self.c = World(self.H, self.W, self.P, _p(self.nonground), _p(self.px), _p(self.py),
                       _p(self.pf), _p(self.pc))

    @property
    def ref(self):
        return C.byref(self.c)


class OracleState:
    """SoA int32/f64 mirror of the device state."""

    def __init__(self, n):
        self.x = np.zeros(n, np.int32)
        self.y = np.zeros(n, np.int32)
        self.fuel = np.zeros(n, np.float64)
        self.cargo = np.zeros(n, np.int32)
        self.origin = np.full(n, -1, np.int32)
        self.dest = np.full(n, -1, np.int32)
        self.reward = np.zeros(n, np.float64)
        self.done = np.zeros(n, np.int32)
        self.err = np.zeros(n, np.int32)
        self.ep_return = np.zeros(n, np.float32)
        self.ep_len = np.zeros(n, np.int32)
        self.n = n

    def fields(self):
        return [_p(self.x), _p(self.y), _p(self.fuel), _p(self.cargo), _p(self.origin), _p(self.dest)]


def step(world, st, *, actions=None, act_type=None, act_a=None, act_b=None, tape=None, seed=0,
         env_id_base=0, t=0):
    if actions is not None:
        mode, ty, a, b = 0, None, np.ascontiguousarray(actions, np.int32), None
    else:
        mode = 1
        ty = np.ascontiguousarray(act_type, np.int32)
        a = np.ascontiguousarray(act_a, np.int32)
        b = np.ascontiguousarray(act_b, np.int32)
    tp = None if tape is None else np.ascontiguousarray(tape, TAPE_DTYPE)
    lib().orc_step_batch(world.ref, st.n, mode, _p(ty), _p(a), _p(b), _p(tp), seed, env_id_base,
                         t, *st.fields(), _p(st.reward), _p(st.done), _p(st.err))


def step_threaded(world, st, actions, pool, threads, *, seed, env_id_base=0, t=0):
    """orc_step_batch (agent-index actions, Philox) over `threads` contiguous slices,
    one per worker of `pool`. ctypes drops the GIL inside the call, so the slices run
    in parallel; slice starts are multiples of 4 (a quad of envs shares its Philox
    blocks), so the result equals one call over all n envs."""
    n = st.n
    per = max(4, (-(-n // threads) + 3) // 4 * 4)
    a = np.ascontiguousarray(actions, np.int32)
    L = lib()

    def run(lo):
        hi = min(n, lo + per)
        sl = slice(lo, hi)
        L.orc_step_batch(world.ref, hi - lo, 0, None, _p(a[sl]), None, None, seed, env_id_base + lo, t,
                         _p(st.x[sl]), _p(st.y[sl]), _p(st.fuel[sl]), _p(st.cargo[sl]),
                         _p(st.origin[sl]), _p(st.dest[sl]), _p(st.reward[sl]), _p(st.done[sl]),
                         _p(st.err[sl]))

    list(pool.map(run, range(0, n, per)))


def step_autoreset(world, st, actions, *, seed, env_id_base=0, t=0, stats=None):
    stats = np.zeros(3, np.float64) if stats is None else stats
    a = np.ascontiguousarray(actions, np.int32)
    rc = lib().orc_step_batch_autoreset(world.ref, st.n, _p(a), seed, env_id_base, t, *st.fields(),
                                        _p(st.ep_return), _p(st.ep_len), _p(st.reward),
                                        _p(st.done), _p(st.err), _p(stats))
    assert rc == 0
    return stats


def reset(world, st, *, mask=None, origin=None, dest=None, seed=0, env_id_base=0, epoch=0):
    m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
    o = None if origin is None else np.ascontiguousarray(origin, np.int32)
    d = None if dest is None else np.ascontiguousarray(dest, np.int32)
    rc = lib().orc_reset_batch(world.ref, st.n, _p(m), _p(o), _p(d), seed, env_id_base, epoch,
                               *st.fields())
    if rc:
        raise ValueError("reset needs at least two ports")


def observe(world, st):
    obs = np.zeros((st.n, 6 + 4 * world.P), np.float32)
    lib().orc_observe(world.ref, st.n, _p(st.x), _p(st.y), _p(st.fuel), _p(st.origin),
                      _p(st.dest), _p(obs))
    return obs


def valid_mask(world, st):
    A = 4 + world.P + 250
    bits = np.zeros((st.n, (A + 7) // 8), np.uint8)
    lib().orc_valid_mask(world.ref, st.n, _p(st.x), _p(st.y), _p(st.origin), _p(bits))
    return bits


def philox(ctr, key):
    c = np.ascontiguousarray(ctr, np.uint32)
    k = np.ascontiguousarray(key, np.uint32)
    out = np.zeros(4, np.uint32)
    lib().orc_philox4x32_10(_p(c), _p(k), _p(out))
    return out


def decode_agent(idx, P):
    """orc_decode_agent: (type, a, b, err) int32 arrays for agent indices idx."""
    idx = np.ascontiguousarray(idx, np.int32)
    out = [np.zeros(len(idx), np.int32) for _ in range(4)]
    lib().orc_decode_agent(int(P), len(idx), idx.ctypes.data, *[o.ctypes.data for o in out])
    return tuple(out)


def gen_actions(n, P, seed, env_id_base=0, t=0):
    out = np.zeros(n, np.int32)
    lib().orc_gen_actions(n, P, seed, env_id_base, t, _p(out))
    return out


def sample_actions(world, st, *, seed, env_id_base=0, t=0):
    """sample_action (environment.py:245-263) per env -> (type, a, b) int32 arrays."""
    ty, a, b = (np.zeros(st.n, np.int32) for _ in range(3))
    lib().orc_sample_actions(world.ref, st.n, *st.fields(), seed, env_id_base, t, _p(ty), _p(a), _p(b))
    return ty, a, b


def rollout(world, st, src, *, max_steps, max_attempts, seed, rollout_base=0):
    """MCTS random rollouts (agents/mcts.py:211-238) -> (ret f64, steps i32, status i32)."""
    s = np.ascontiguousarray(src, np.int32)
    m = len(s)
    ret = np.zeros(m, np.float64)
    steps = np.zeros(m, np.int32)
    status = np.zeros(m, np.int32)
    lib().orc_rollout(world.ref, st.n, *st.fields(), m, _p(s), max_steps, max_attempts, seed,
                      rollout_base, _p(ret), _p(steps), _p(status))
    return ret, steps, status


def feistel_perm(p, D, key):
    k = np.ascontiguousarray(key, np.uint32)
    return int(lib().orc_feistel_perm(p, D, _p(k)))


def replay_pick(size, batch, invalid, *, seed, t):
    """update()'s minibatch indices (agents/dqn.py:213) under the sampler contract."""
    inv = np.ascontiguousarray(invalid, np.uint8)
    assert len(inv) >= size
    slot = np.zeros(batch, np.int64)
    lib().orc_replay_pick(size, batch, _p(inv), seed, t, _p(slot))
    return slot


class ReplayMemory:
    """DQNAgent.memory (agents/dqn.py:86, :117-123) as the reference keeps it: a FIFO of
    (preprocess_state row, action, reward, next row, done) of capacity `maxlen`, as
    numpy rows, here in ring order (slot = push index mod maxlen) so that indices
    line up with the device ring. `invalid` marks transitions whose step raised (the
    reference never stores them; the device ring keeps them flagged)."""

    def __init__(self, maxlen, width):
        self.maxlen, self.size, self.head = maxlen, 0, 0
        self.obs = np.zeros((maxlen, width), np.float32)
        self.next_obs = np.zeros((maxlen, width), np.float32)
        self.act = np.zeros(maxlen, np.int64)
        self.rew = np.zeros(maxlen, np.float32)
        self.done = np.zeros(maxlen, np.float32)
        self.invalid = np.zeros(maxlen, np.uint8)

    def push(self, obs, act, rew, next_obs, done, invalid):
        for i in range(len(act)):
            s = self.head
            self.obs[s], self.next_obs[s] = obs[i], next_obs[i]
            self.act[s], self.rew[s], self.done[s] = act[i], rew[i], float(bool(done[i]))
            self.invalid[s] = 1 if invalid[i] else 0
            self.head = (self.head + 1) % self.maxlen
        self.size = min(self.size + len(act), self.maxlen)

    def sample(self, batch, *, seed, t):
        """-> obs, next_obs, act, rew, done, weight exactly as se_replay_sample writes them."""
        slot = replay_pick(self.size, batch, self.invalid, seed=seed, t=t)
        ok = slot >= 0
        s = np.where(ok, slot, 0)
        w = self.obs.shape[1]
        z = np.zeros(w, np.float32)
        obs = np.where(ok[:, None], self.obs[s], z)
        nxt = np.where(ok[:, None], self.next_obs[s], z)
        return (obs, nxt, np.where(ok, self.act[s], 0), np.where(ok, self.rew[s], 0).astype(np.float32),
                np.where(ok, self.done[s], 0).astype(np.float32), ok.astype(np.float32))
