"""One environment on the host behind shipping.Environment (the default stepper).

The reference steps one env per call (agents/dqn.py:287, agents/mcts.py:228-236). On the
GPU that is a launch plus a stream synchronise per step, ~18 us, where the reference's
Python step takes ~10 us. The host stepper runs the step kernels' own per-env code
(``replay_env`` in csrc/shipenv.hip, compiled for the host: se_host_step_replay) on an
88-byte state block in host memory: one C call per step, no device. It is not a
fallback: the library is the same, a missing library still raises
NativeLibraryError, and ``SHIPENV_STEPPER=gpu`` selects the kernel (DeviceStepper).
tests/test_compat_gpu.py checks both steppers give the same bits on every golden tape
and seeded reference trace.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .. import _native as N
from ._device import _IN, _OUT, _RESET_OUT, StepResult

# the block: one env's SoA fields (se_state pointers), its typed action and its tape
#   0 x u8, 1 y u8, 2 origin u8, 3 dest u8, 4 done u8, 5 err i8, 8 fuel f64, 16 cargo i32,
#   20 reward f32, 24 reward64 f64, 32 type i32, 36 a i32, 40 b i32,
#   48 tape {u_fuel, u_gate, u_type, beta f64; arrive_dest, used i32}
_SIZE = 88  # the structs (shared with the GPU stepper's se_server_block, whose first 88 bytes this is)
_I32_MIN, _I32_MAX = -(2 ** 31), 2 ** 31 - 1
_NONE = N.SE_NONE


def _clamp32(v):
    return _I32_MIN if v < _I32_MIN else (_I32_MAX if v > _I32_MAX else v)


class HostStepper:
    def __init__(self, water, port_x, port_y, port_fuel, port_cargo):
        lib = N.lib()
        self._lib = lib
        self._buf = np.zeros(_SIZE + 16, np.uint8)
        off = (-self._buf.ctypes.data) % 16
        self.block = self._buf[off:off + _SIZE]
        self._mv = memoryview(self.block)
        b = self.block.ctypes.data
        self._state = N.SeState(b + 0, b + 1, b + 8, b + 16, b + 2, b + 3, b + 20, b + 4, b + 5,
                                None, None, None, None, b + 24)
        self._sp = C.addressof(self._state)
        self._args = (b + 32, b + 36, b + 40, b + 48)
        self._origin = np.zeros(1, np.int32)
        self._dest = np.zeros(1, np.int32)
        self._h = C.c_void_p()
        self._make(water, port_x, port_y, port_fuel, port_cargo)

    def _make(self, water, port_x, port_y, port_fuel, port_cargo):
        h = _create(self._lib, water, port_x, port_y, port_fuel, port_cargo)
        self.close()
        self._h = h
        self._hv = h.value

    def set_world(self, water, port_x, port_y, port_fuel, port_cargo):
        """Replace map and ports (a new host world: the map size may change)."""
        self._make(water, port_x, port_y, port_fuel, port_cargo)

    def step(self, x, y, fuel, cargo, origin, dest, act_type, a, b, tape):
        """tape: (u_fuel, u_gate, u_type, beta, arrive_dest), NaN / -1 where not drawn."""
        _IN.pack_into(self._mv, 0, x, y, _NONE if origin is None else origin, _NONE if dest is None else dest,
                      fuel, cargo, act_type, _clamp32(a), _clamp32(b),
                      tape[0], tape[1], tape[2], tape[3], tape[4])
        ta, aa, ba, tp = self._args
        rc = self._lib.se_host_step_replay(self._hv, 1, self._sp, ta, aa, ba, tp)
        if rc:
            N.check(rc)
        x, y, org, dst, done, err, fuel, cargo, _, r64, used = _OUT.unpack_from(self._mv, 0)
        return StepResult(x, y, fuel, cargo, -1 if org == _NONE else org, -1 if dst == _NONE else dst,
                          r64, bool(done), err, used)

    def reset_to(self, origin, dest):
        self._origin[0], self._dest[0] = origin, dest
        N.check(self._lib.se_host_reset_to(self._hv, 1, self._sp, None, self._origin.ctypes.data,
                                           self._dest.ctypes.data))
        x, y, org, dst, fuel, cargo = _RESET_OUT.unpack_from(self._mv, 0)
        return StepResult(x, y, fuel, cargo, org, dst, 0.0, False, 0, 0)

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.se_host_destroy(self._h)
            self._h = C.c_void_p()
            self._hv = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


def host_step_replay(water, port_x, port_y, port_fuel, port_cargo, state, act_type, a, b, tape):
    """se_host_step_replay over n host envs at once (numpy): state is a dict of SoA arrays
    x, y, origin, dest (u8, 255 = None), fuel (f64), cargo (i32); tape a TAPE_DTYPE array.
    Returns the post-step state dict plus reward (f32), reward64, done, err and tape
    (with `used`). The inputs are not modified."""
    from ..vec import TAPE_DTYPE

    lib = N.lib()
    n = len(act_type)
    st = {k: np.array(state[k], dtype=dt) for k, dt in
          (("x", np.uint8), ("y", np.uint8), ("origin", np.uint8), ("dest", np.uint8),
           ("fuel", np.float64), ("cargo", np.int32))}
    out = {"reward": np.zeros(n, np.float32), "reward64": np.zeros(n, np.float64),
           "done": np.zeros(n, np.uint8), "err": np.zeros(n, np.int8)}
    tp = np.array(tape, dtype=TAPE_DTYPE)
    ty, aa, bb = (np.ascontiguousarray(v, np.int32) for v in (act_type, a, b))
    ptr = lambda v: v.ctypes.data  # noqa: E731
    s = N.SeState(ptr(st["x"]), ptr(st["y"]), ptr(st["fuel"]), ptr(st["cargo"]), ptr(st["origin"]),
                  ptr(st["dest"]), ptr(out["reward"]), ptr(out["done"]), ptr(out["err"]), None, None, None,
                  None, ptr(out["reward64"]))
    h = _create(lib, water, port_x, port_y, port_fuel, port_cargo)
    try:
        N.check(lib.se_host_step_replay(h, n, C.byref(s), ptr(ty), ptr(aa), ptr(bb), ptr(tp)))
    finally:
        lib.se_host_destroy(h)
    return st | out | {"tape": tp}


def host_reset_to(water, port_x, port_y, port_fuel, port_cargo, origin, dest):
    """se_host_reset_to over n host envs: the post-reset state dict."""
    lib = N.lib()
    o, d = np.ascontiguousarray(origin, np.int32), np.ascontiguousarray(dest, np.int32)
    n = len(o)
    st = {"x": np.zeros(n, np.uint8), "y": np.zeros(n, np.uint8), "origin": np.zeros(n, np.uint8),
          "dest": np.zeros(n, np.uint8), "fuel": np.zeros(n, np.float64), "cargo": np.ones(n, np.int32),
          "reward": np.ones(n, np.float32), "done": np.ones(n, np.uint8), "err": np.ones(n, np.int8)}
    ptr = lambda v: v.ctypes.data  # noqa: E731
    s = N.SeState(*[ptr(st[k]) for k in ("x", "y", "fuel", "cargo", "origin", "dest", "reward", "done", "err")],
                  None, None, None, None, None)
    h = _create(lib, water, port_x, port_y, port_fuel, port_cargo)
    try:
        N.check(lib.se_host_reset_to(h, n, C.byref(s), None, ptr(o), ptr(d)))
    finally:
        lib.se_host_destroy(h)
    return st


def _create(lib, water, port_x, port_y, port_fuel, port_cargo):
    water = np.ascontiguousarray(water, np.uint8)
    H, W = water.shape
    px, py, pf, pc = (np.ascontiguousarray(v, np.int32) for v in (port_x, port_y, port_fuel, port_cargo))
    h = C.c_void_p()
    N.check(lib.se_host_create(C.byref(h), H, W, water.ctypes.data_as(C.c_void_p), len(px),
                               px.ctypes.data_as(C.c_void_p), py.ctypes.data_as(C.c_void_p),
                               pf.ctypes.data_as(C.c_void_p), pc.ctypes.data_as(C.c_void_p)))
    return h
