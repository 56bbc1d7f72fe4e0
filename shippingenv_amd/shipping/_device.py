"""One environment on the GPU behind shipping.Environment.

The compat class keeps the reference's attributes on the host (agents read and
assign them directly) and runs every state transition through the step kernel's
per-env code: se_step_replay's work on a one-env handle whose SoA buffers, action
and tape all live in one 256-byte block of coherent pinned host memory
(se_host_alloc), which the GPU reads and writes in place (ROCm maps pinned host
memory into the GPU's address space). No copies: an H2D and a D2H copy per step
measured 38.8 us per step for config 1, BASELINE configs[0].

By default a step is one call to the resident stepper wave (se_server_call,
csrc/server.h): the wave polls a mailbox after the block and answers each command,
so a step costs no launch and no stream synchronise. SHIPENV_GPU_SERVER=0 (or
server=False) steps with one se_step_replay launch and one synchronise instead.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np
import torch

from .. import _native as N
from ..vec import _raw_stream

_hip = None


def _hip_sync(stream):
    """hipStreamSynchronize on a raw stream handle: torch's Stream object costs a few
    microseconds per step to build, a third of the N = 1 step's host time."""
    global _hip
    if _hip is None:
        _hip = C.CDLL("libamdhip64.so")  # already loaded by torch
        _hip.hipStreamSynchronize.argtypes = [C.c_void_p]
        _hip.hipStreamSynchronize.restype = C.c_int
    rc = _hip.hipStreamSynchronize(stream)
    if rc != 0:
        raise N.NativeLibraryError(f"hipStreamSynchronize failed ({rc})")

# byte offsets inside the I/O block (each field 16-byte aligned for se_bind)
_X, _Y, _ORG, _DST, _DONE, _ERR = 0, 16, 32, 48, 64, 80
_FUEL, _CARGO, _REW, _REW64 = 96, 112, 128, 144
_TYPE, _A, _B, _TAPE = 160, 176, 192, 208
_MBOX = 256  # the stepper wave's mailbox: 4 u32 (csrc/server.h)
_SIZE = 272
_I32_MIN, _I32_MAX = -(2 ** 31), 2 ** 31 - 1


@dataclass
class StepResult:
    x: int
    y: int
    fuel: float
    cargo: int
    origin: int  # -1 = None
    dest: int  # -1 = None
    reward: float  # the reference's f64 reward
    done: bool
    err: int
    used: int  # SE_USED_* bits


def _clamp32(v):
    return _I32_MIN if v < _I32_MIN else (_I32_MAX if v > _I32_MAX else v)


class DeviceStepper:
    def __init__(self, water, port_x, port_y, port_fuel, port_cargo, device=None, server=None):
        if not torch.cuda.is_available():
            raise N.NativeLibraryError("shipping.Environment steps on a ROCm GPU; none is visible")
        lib = N.lib()
        self.dev = torch.device("cuda", torch.cuda.current_device()) if device is None \
            else torch.device(device)
        if server is None:
            server = os.environ.get("SHIPENV_GPU_SERVER", "1").strip() != "0"
        self.server = bool(server)
        blk = C.c_void_p()
        with torch.cuda.device(self.dev):  # pinned for (mapped into) this GPU
            N.check(lib.se_host_alloc(_SIZE, C.byref(blk)))
        self._blk = blk
        self.h = np.ctypeslib.as_array((C.c_uint8 * _SIZE).from_address(blk.value))
        water = np.ascontiguousarray(water, np.uint8)
        H, W = water.shape
        self._h = C.c_void_p()
        px, py, pf, pc = (np.ascontiguousarray(v, np.int32) for v in (port_x, port_y, port_fuel, port_cargo))
        with torch.cuda.device(self.dev):
            N.check(lib.se_create(C.byref(self._h), self.dev.index, 1, 0, H, W,
                                  water.ctypes.data_as(C.c_void_p), len(px),
                                  px.ctypes.data_as(C.c_void_p), py.ctypes.data_as(C.c_void_p),
                                  pf.ctypes.data_as(C.c_void_p), pc.ctypes.data_as(C.c_void_p), 0, 0))
        b = blk.value
        self._state = N.SeState(b + _X, b + _Y, b + _FUEL, b + _CARGO, b + _ORG, b + _DST,
                                b + _REW, b + _DONE, b + _ERR, None, None, None, None, b + _REW64)
        N.check(lib.se_bind(self._h, C.byref(self._state)))
        self._base = b
        self._srv = C.c_void_p()
        if self.server:
            N.check(lib.se_server_create(C.byref(self._srv), self._h, b, _MBOX, b + _TYPE, b + _A, b + _B,
                                         b + _TAPE, b + _MBOX))
        self._f64 = self.h.view(np.float64)
        self._i32 = self.h.view(np.int32)

    def _put_state(self, x, y, fuel, cargo, origin, dest):
        h = self.h
        h[_X], h[_Y] = x, y
        h[_ORG] = N.SE_NONE if origin is None else origin
        h[_DST] = N.SE_NONE if dest is None else dest
        self._f64[_FUEL // 8] = fuel
        self._i32[_CARGO // 4] = cargo

    def _get(self, err, used):
        h = self.h
        org, dst = int(h[_ORG]), int(h[_DST])
        return StepResult(int(h[_X]), int(h[_Y]), float(self._f64[_FUEL // 8]),
                          int(self._i32[_CARGO // 4]), -1 if org == N.SE_NONE else org,
                          -1 if dst == N.SE_NONE else dst, float(self._f64[_REW64 // 8]),
                          bool(h[_DONE]), err, used)

    def set_world(self, water, port_x, port_y, port_fuel, port_cargo):
        """Replace map and ports (a new handle: the map size may change)."""
        self.close()
        self.__init__(water, port_x, port_y, port_fuel, port_cargo, self.dev, self.server)

    def step(self, x, y, fuel, cargo, origin, dest, act_type, a, b, tape):
        """tape: (u_fuel, u_gate, u_type, beta, arrive_dest), NaN / -1 where not drawn."""
        self._put_state(x, y, fuel, cargo, origin, dest)
        i32 = self._i32
        i32[_TYPE // 4], i32[_A // 4], i32[_B // 4] = act_type, _clamp32(a), _clamp32(b)
        f = self._f64
        t0 = _TAPE // 8
        f[t0], f[t0 + 1], f[t0 + 2], f[t0 + 3] = tape[0], tape[1], tape[2], tape[3]
        i32[_TAPE // 4 + 8], i32[_TAPE // 4 + 9] = tape[4], 0
        self._f64[_REW64 // 8] = 0.0
        if self._srv.value:
            N.check(N.lib().se_server_call(self._srv, N.SERVER_STEP))  # answered: results in the block
        else:
            b_ = self._base
            stream = _raw_stream(self.dev.index)
            N.check(N.lib().se_step_replay(self._h, b_ + _TYPE, b_ + _A, b_ + _B, b_ + _TAPE, stream))
            _hip_sync(stream)  # the kernel wrote its results into the pinned block
        return self._get(int(self.h[_ERR].astype(np.int8)), int(i32[_TAPE // 4 + 9]))

    def reset_to(self, origin, dest):
        i32 = self._i32
        i32[_TYPE // 4], i32[_A // 4] = origin, dest
        if self._srv.value:
            N.check(N.lib().se_server_call(self._srv, N.SERVER_RESET_TO))
        else:
            b_ = self._base
            stream = _raw_stream(self.dev.index)
            N.check(N.lib().se_reset_to(self._h, None, b_ + _TYPE, b_ + _A, stream))
            _hip_sync(stream)
        return self._get(0, 0)

    def launches(self):
        """Kernel launches of the stepper wave so far (1 + restarts after idle exits)."""
        n = C.c_uint64()
        N.check(N.lib().se_server_launches(self._srv, C.byref(n)))
        return int(n.value)

    def close(self):
        lib = N.lib()
        if getattr(self, "_srv", None) is not None and self._srv.value:
            lib.se_server_destroy(self._srv)  # ends the wave
            self._srv = C.c_void_p()
        if getattr(self, "_h", None) is not None and self._h.value:
            torch.cuda.synchronize(self.dev)
            lib.se_destroy(self._h)
            self._h = C.c_void_p()
        if getattr(self, "_blk", None) is not None and self._blk.value:
            lib.se_host_free(self._blk)
            self._blk = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass
