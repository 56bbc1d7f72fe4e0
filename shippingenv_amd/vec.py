"""VecEnv: N ShippingEnv environments stepped together on one MI355X.

The batched form of shipping.Environment (shipping/environment.py:28-376).
State lives in HBM as SoA torch tensors owned by this object and bound once
to the native handle (include/shipenv.h, se_bind); every call launches on the
current torch stream and returns without synchronising the host.

Field widths (DESIGN.md "Data layout"): x, y, origin, dest u8 (origin/dest
255 = None), fuel f64, cargo i32, reward f32, done u8, err i8.
"""
from __future__ import annotations

import ctypes as C
import random as _random

import numpy as np
import torch

from . import _native as N
from .maps import builtin_water

DEFAULT_PORTS = [[41, 40], [60, 22], [78, 29], [49, 72], [62, 72]]  # utils/constants.py:57-63

TAPE_DTYPE = np.dtype(
    [("u_fuel", "<f8"), ("u_gate", "<f8"), ("u_type", "<f8"), ("beta", "<f8"),
     ("arrive_dest", "<i4"), ("used", "<i4")]
)  # se_tape


def draw_port_stocks(n_ports, seed):
    """add_port's stocks (environment.py:63-64): randint(5, 20) for fuel, then cargo, per port."""
    rng = _random.Random(seed)
    fuel, cargo = [], []
    for _ in range(n_ports):
        fuel.append(rng.randint(5, 20))
        cargo.append(rng.randint(5, 20))
    return fuel, cargo


def random_water_ports(water, n_ports, seed):
    """n distinct water cells, seeded (config 4's 64 random ports)."""
    rng = np.random.default_rng(seed)
    cells = np.argwhere(np.asarray(water) != 0)
    pick = rng.choice(len(cells), size=n_ports, replace=False)
    return [[int(a), int(b)] for a, b in cells[np.sort(pick)]]


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


try:  # the current stream's hipStream_t without building a torch Stream object
    _get_raw_stream = torch._C._cuda_getCurrentRawStream
except AttributeError:  # pragma: no cover - older torch
    _get_raw_stream = None


def _raw_stream(index):
    if _get_raw_stream is not None:
        return _get_raw_stream(index)
    return torch.cuda.current_stream(index).cuda_stream


def _i32(a):
    return np.ascontiguousarray(a, np.int32)


class VecEnv:
    def __init__(self, n, *, water=None, ports=None, port_fuel=None, port_cargo=None, seed=0,
                 env_id_base=0, device=None, auto_reset=False, stock_seed=None):
        if not torch.cuda.is_available():
            raise N.NativeLibraryError("VecEnv needs a ROCm GPU (torch.cuda.is_available() is False)")
        lib = N.lib()
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None \
            else torch.device(device)
        self.n = int(n)
        self.seed = int(seed)
        self.env_id_base = int(env_id_base)
        self.auto_reset = bool(auto_reset)
        self.water = np.ascontiguousarray(builtin_water() if water is None else water, np.uint8)
        self.H, self.W = self.water.shape
        ports = DEFAULT_PORTS if ports is None else ports
        if port_fuel is None or port_cargo is None:
            f, c = draw_port_stocks(len(ports), self.seed if stock_seed is None else stock_seed)
            port_fuel = f if port_fuel is None else port_fuel
            port_cargo = c if port_cargo is None else port_cargo
        self.port_x = _i32([p[0] for p in ports])
        self.port_y = _i32([p[1] for p in ports])
        self.port_fuel = _i32(port_fuel)
        self.port_cargo = _i32(port_cargo)
        self.P = len(self.port_x)

        kw = dict(device=self.device)
        n = self.n
        self.x = torch.zeros(n, dtype=torch.uint8, **kw)
        self.y = torch.zeros(n, dtype=torch.uint8, **kw)
        self.fuel = torch.zeros(n, dtype=torch.float64, **kw)
        self.cargo = torch.zeros(n, dtype=torch.int32, **kw)
        self.origin = torch.full((n,), N.SE_NONE, dtype=torch.uint8, **kw)
        self.dest = torch.full((n,), N.SE_NONE, dtype=torch.uint8, **kw)
        self.reward = torch.zeros(n, dtype=torch.float32, **kw)
        self.done = torch.zeros(n, dtype=torch.uint8, **kw)
        self.err = torch.zeros(n, dtype=torch.int8, **kw)
        self.ep_return = torch.zeros(n, dtype=torch.float32, **kw)
        # episode-start stamps on the step counter (include/shipenv.h se_state.ep_start);
        # the running lengths are the property ep_len
        self.ep_start = torch.zeros(n, dtype=torch.int32, **kw)
        self._h = C.c_void_p()
        flags = N.SE_FLAG_AUTO_RESET if self.auto_reset else 0
        with torch.cuda.device(self.device):
            N.check(lib.se_create(C.byref(self._h), self.device.index, n, self.env_id_base,
                                  self.H, self.W, self.water.ctypes.data_as(C.c_void_p), self.P,
                                  self.port_x.ctypes.data_as(C.c_void_p),
                                  self.port_y.ctypes.data_as(C.c_void_p),
                                  self.port_fuel.ctypes.data_as(C.c_void_p),
                                  self.port_cargo.ctypes.data_as(C.c_void_p), self.seed, flags))
        # done lists (auto-reset): per-wave segments, double-buffered
        # (include/shipenv.h se_done_layout); records are {env, ep_return bits, ep_len, step}
        seg, nseg = C.c_int64(), C.c_int32()
        N.check(lib.se_done_layout(self._h, C.byref(seg), C.byref(nseg)))
        self.done_seg, self.done_segments = seg.value, nseg.value
        nrec = 2 * self.done_seg * self.done_segments if self.auto_reset else 1
        self.done_recs = torch.zeros((nrec, 4), dtype=torch.int32, **kw)
        self.done_count = torch.zeros(max(2 * self.done_segments, 4), dtype=torch.int32, **kw)
        self._done_out = None
        self._state = N.SeState(*[t.data_ptr() for t in (
            self.x, self.y, self.fuel, self.cargo, self.origin, self.dest, self.reward,
            self.done, self.err, self.ep_return, self.ep_start, self.done_recs, self.done_count)] + [None])
        N.check(lib.se_bind(self._h, C.byref(self._state)))
        self._se_step = lib.se_step
        self._se_step_seq = lib.se_step_seq
        self._dev_index = self.device.index
        self._stats = torch.zeros(3, dtype=torch.float64, **kw)

    # ------------------------------------------------------------------ helpers
    @property
    def action_space_size(self):
        """utils/preprocessing.py:93-108: 4 moves + P ports + 50 cargo + 200 fuel amounts."""
        return 4 + self.P + 50 + 200

    @property
    def obs_size(self):
        return 6 + 4 * self.P

    @property
    def ep_len(self):
        """Running episode lengths in step calls (auto-reset): (step counter - ep_start)
        mod 2^32, as a new int32 device tensor computed on the current stream. A snapshot:
        a reference to it does not follow later steps (read the property again). Without
        auto-reset the stamps are only written by reset (se_reset stamps the counter), so
        the value is the steps since the last reset."""
        t = self.counters[0] & 0xFFFFFFFF
        d = (t - self.ep_start.to(torch.int64)) & 0xFFFFFFFF
        return torch.where(d >= 2**31, d - 2**32, d).to(torch.int32)

    def _stream(self):
        return C.c_void_p(_raw_stream(self._dev_index))

    def _dev(self, t, dtype, count=None):
        """A contiguous, 16-byte aligned device tensor of `count` (default n) entries."""
        if not isinstance(t, torch.Tensor):
            t = torch.as_tensor(np.asarray(t), device=self.device)
        t = t.to(device=self.device, dtype=dtype)
        if not t.is_contiguous() or t.data_ptr() % 16:
            t = t.contiguous().clone()
        want = self.n if count is None else count
        if t.numel() != want:
            raise ValueError(f"expected {want} entries, got {t.numel()}")
        return t

    # ------------------------------------------------------------------ API
    def set_ports(self, ports, port_fuel, port_cargo):
        self.port_x = _i32([p[0] for p in ports])
        self.port_y = _i32([p[1] for p in ports])
        self.port_fuel = _i32(port_fuel)
        self.port_cargo = _i32(port_cargo)
        self.P = len(self.port_x)
        N.check(N.lib().se_set_ports(self._h, self.P, self.port_x.ctypes.data_as(C.c_void_p),
                                     self.port_y.ctypes.data_as(C.c_void_p),
                                     self.port_fuel.ctypes.data_as(C.c_void_p),
                                     self.port_cargo.ctypes.data_as(C.c_void_p)))

    def reset(self, mask=None):
        """reset() (environment.py:227-243) of every env, or of those with mask != 0."""
        m = None if mask is None else self._dev(mask, torch.uint8)
        N.check(N.lib().se_reset(self._h, _ptr(m), self._stream()))
        self._keep = m

    def reset_to(self, origin, dest, mask=None):
        o, d = self._dev(origin, torch.int32), self._dev(dest, torch.int32)
        m = None if mask is None else self._dev(mask, torch.uint8)
        N.check(N.lib().se_reset_to(self._h, _ptr(m), _ptr(o), _ptr(d), self._stream()))
        self._keep = (o, d, m)

    def step(self, actions):
        """step() with int32 actions in the agent-index encoding; returns (reward, done, err).

        The per-call host path is kept short (it is a few microseconds against a
        ~10 us kernel at N = 2^20): an int32, contiguous, aligned device tensor of n
        entries goes straight to se_step."""
        a = actions
        if not (type(a) is torch.Tensor and a.dtype is torch.int32 and a.is_cuda
                and a.get_device() == self._dev_index and a.is_contiguous() and a.numel() == self.n
                and a.data_ptr() % 16 == 0):
            a = self._dev(actions, torch.int32)
        rc = self._se_step(self._h, a.data_ptr(), _raw_stream(self._dev_index))
        if rc:
            N.check(rc)
        self._keep = a
        return self.reward, self.done, self.err

    def step_seq(self, actions, mark=None, mark_after=0):
        """len(actions) consecutive step() calls issued from native code (se_step_seq):
        actions is an int32 device tensor [K, n] (rows contiguous, 16-byte aligned), row k
        the actions of step k. mark: a torch.cuda.Event recorded on the current stream right
        after launch `mark_after` (se_step_seq_mark; 0 = before launch 1, the timed loop's
        form; at most K), a timer mark inside the one native call. Returns the last
        step's (reward, done, err)."""
        a = actions
        if not (type(a) is torch.Tensor and a.dtype is torch.int32 and a.is_cuda and a.dim() == 2
                and a.get_device() == self._dev_index and a.shape[1] == self.n and a.stride(1) == 1
                and a.data_ptr() % 16 == 0 and (a.shape[0] < 2 or a.stride(0) % 4 == 0 or self.n == 0)):
            raise ValueError("step_seq needs an int32 [K, n] device tensor with 16-byte aligned rows")
        ld = a.stride(0) if self.n else 0  # an empty batch: no rows to stride over
        if mark is not None:
            if mark.cuda_event == 0:  # torch creates the HIP event on its first record
                with torch.cuda.device(self.device):
                    mark.record()
            ev_dev = getattr(mark, "device", None)
            if ev_dev is not None and ev_dev.index is not None and ev_dev.index != self._dev_index:
                raise ValueError(f"mark event is on {ev_dev}, the env on cuda:{self._dev_index}")
            if not 0 <= int(mark_after) <= a.shape[0]:
                raise ValueError(f"mark_after must be in [0, {a.shape[0]}], got {mark_after}")
            rc = N.lib().se_step_seq_mark(self._h, a.data_ptr(), ld, a.shape[0],
                                          _raw_stream(self._dev_index), mark.cuda_event, int(mark_after))
            if rc:
                N.check(rc)
            self._keep = a
            return self.reward, self.done, self.err
        rc = self._se_step_seq(self._h, a.data_ptr(), ld, a.shape[0], _raw_stream(self._dev_index))
        if rc:
            N.check(rc)
        self._keep = a
        return self.reward, self.done, self.err

    def step_typed(self, act_type, a, b):
        t, aa, bb = (self._dev(v, torch.int32) for v in (act_type, a, b))
        N.check(N.lib().se_step_typed(self._h, _ptr(t), _ptr(aa), _ptr(bb), self._stream()))
        self._keep = (t, aa, bb)
        return self.reward, self.done, self.err

    def step_replay(self, act_type, a, b, tape):
        """step() with recorded variates; tape: numpy structured array of TAPE_DTYPE (n,)."""
        t, aa, bb = (self._dev(v, torch.int32) for v in (act_type, a, b))
        tape = np.ascontiguousarray(tape, TAPE_DTYPE)
        if len(tape) != self.n:
            raise ValueError("tape length != n")
        tp = torch.from_numpy(tape.view(np.uint8).reshape(-1).copy()).to(self.device)
        N.check(N.lib().se_step_replay(self._h, _ptr(t), _ptr(aa), _ptr(bb), _ptr(tp),
                                       self._stream()))
        self._keep = (t, aa, bb, tp)
        return self.reward, self.done, self.err

    def step_agent_replay(self, actions, tape):
        """se_step_agent_replay: agent-index actions (the se_step encoding) with the
        reference's draws from tape (numpy TAPE_DTYPE, n): the production agent-path
        kernel in its replay-tape instantiation (parity). Returns (reward, done, err,
        tape with `used` filled in)."""
        a = self._dev(actions, torch.int32)
        tape = np.ascontiguousarray(tape, TAPE_DTYPE)
        if len(tape) != self.n:
            raise ValueError("tape length != n")
        tp = torch.from_numpy(tape.view(np.uint8).reshape(-1).copy()).to(self.device)
        N.check(N.lib().se_step_agent_replay(self._h, _ptr(a), _ptr(tp), self._stream()))
        self._keep = (a, tp)
        used = tp.cpu().numpy().view(TAPE_DTYPE)
        return self.reward, self.done, self.err, used

    def observe(self, out=None):
        """preprocess_state rows (utils/preprocessing.py:25-62) as f32 [n, 6+4P]."""
        if out is None:
            out = torch.empty((self.n, self.obs_size), dtype=torch.float32, device=self.device)
        N.check(N.lib().se_observe(self._h, _ptr(out), out.stride(0), self._stream()))
        return out

    def valid_mask(self, out=None):
        """DQN is_valid_action bits (agents/dqn.py:125-175), packed MSB-first per row."""
        stride = (self.action_space_size + 7) // 8
        if out is None:
            out = torch.empty((self.n, stride), dtype=torch.uint8, device=self.device)
        N.check(N.lib().se_valid_mask(self._h, _ptr(out), self._stream()))
        return out

    def gen_actions(self, t, out=None):
        """The bench's synthetic agent (config 3/4 action mix) for step index t."""
        if out is None:
            out = torch.empty(self.n, dtype=torch.int32, device=self.device)
        N.check(N.lib().se_gen_actions(self._h, _ptr(out), int(t) & 0xFFFFFFFF, self._stream()))
        return out

    def sample_actions(self, t, out=None):
        """sample_action() (environment.py:245-263) of every env as typed actions
        (type, a, b) int32 tensors for step_typed; type < 0 where the reference raises
        (SAMPLE_RAISES) or never returns (SAMPLE_NO_OTHER_PORT). t selects the draw."""
        if out is None:
            out = tuple(torch.empty(self.n, dtype=torch.int32, device=self.device) for _ in range(3))
        ty, a, b = out
        N.check(N.lib().se_sample_actions(self._h, _ptr(ty), _ptr(a), _ptr(b),
                                          int(t) & 0xFFFFFFFF, self._stream()))
        return ty, a, b

    def rollout(self, src, max_steps=100, max_attempts=None, rollout_base=0):
        """MCTS random rollouts (agents/mcts.py:211-238) from copies of envs src (int32 [m]):
        returns (ret f64, steps i32, status i32) device tensors; env state is untouched.
        max_attempts bounds the reference's unbounded retry of raising steps (default
        8 * max_steps). Rollout r draws from Philox(seed, rollout_base + r): pass fresh
        bases for independent rollouts."""
        if not isinstance(src, torch.Tensor):
            src = torch.as_tensor(np.asarray(src))
        m = src.numel()
        s = self._dev(src, torch.int32, count=m)
        if max_attempts is None:
            max_attempts = 8 * max_steps
        ret = torch.empty(m, dtype=torch.float64, device=self.device)
        steps = torch.empty(m, dtype=torch.int32, device=self.device)
        status = torch.empty(m, dtype=torch.int32, device=self.device)
        N.check(N.lib().se_rollout(self._h, _ptr(s), m, int(max_steps), int(max_attempts),
                                   int(rollout_base), _ptr(ret), _ptr(steps), _ptr(status),
                                   self._stream()))
        self._keep = s
        return ret, steps, status

    def episode_stats(self):
        """Device f64[3] {sum of returns, episodes, sum of lengths} since the last clear."""
        N.check(N.lib().se_episode_stats(self._h, _ptr(self._stats), self._stream()))
        return self._stats

    def clear_stats(self):
        N.check(N.lib().se_clear_stats(self._h, self._stream()))

    def done_list(self):
        """Episodes finished by the last step (auto-reset), in env order:
        (env, ep_return, ep_len, step) tensors."""
        if self._done_out is None:
            self._done_out = torch.empty((self.n + 4, 4), dtype=torch.int32, device=self.device)
            self._done_cnt = torch.empty(1, dtype=torch.int32, device=self.device)
        N.check(N.lib().se_done_compact(self._h, _ptr(self._done_out), _ptr(self._done_cnt),
                                        self._stream()))
        k = int(self._done_cnt.item())
        raw = self._done_out[:k].clone()
        return raw[:, 0], raw[:, 1].view(torch.float32), raw[:, 2], raw[:, 3]

    @property
    def counters(self):
        s, e = C.c_uint64(), C.c_uint64()
        N.check(N.lib().se_get_counters(self._h, C.byref(s), C.byref(e)))
        return s.value, e.value

    def set_counters(self, step, epoch):
        N.check(N.lib().se_set_counters(self._h, int(step), int(epoch)))

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            torch.cuda.synchronize(self.device)
            N.lib().se_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass
