"""One environment on the GPU behind shipping.Environment.

The compat class keeps the reference's attributes on the host (agents read and
assign them directly) and runs every state transition through the step kernels'
per-env code on the GPU. The env's state, its typed action and its tape are one
se_server_block (include/shipenv.h) in coherent pinned host memory (se_host_alloc),
which the GPU reads and writes in place (ROCm maps pinned host memory into the GPU's
address space); the inputs go in with one struct.pack_into and the results come out
with one unpack_from, as in the host stepper. No copies: an H2D and a D2H copy per
step measured 38.8 us per step for config 1, BASELINE configs[0].

By default a step is one call to the resident stepper wave (se_server_call,
csrc/server.h): the wave polls the block and answers each command, so a step costs
no launch and no stream synchronise. SHIPENV_GPU_SERVER=0 (or server=False) steps
with one se_step_replay launch and one synchronise instead.
"""
from __future__ import annotations

import ctypes as C
import os
import struct
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

# the block: se_server_block (include/shipenv.h), 128 bytes in coherent pinned host memory;
# bytes 0-87 are also shipping/_host.py's block layout:
#   0 x u8, 1 y u8, 2 origin u8, 3 dest u8, 4 done u8, 5 err i8, 8 fuel f64, 16 cargo i32,
#   20 reward f32, 24 reward64 f64, 32 type i32, 36 a i32, 40 b i32, 44 seq0 (the wave's),
#   48 tape {u_fuel, u_gate, u_type, beta f64; arrive_dest, used i32}, 88.. the mailbox
# The launch path (se_bind and se_step_replay want 16-byte aligned buffers) binds the handle
# to a layout of 16-byte aligned fields from byte 256 (_L) and copies through it.
_IN = struct.Struct("<4B4xdi12xiii4xddddi")          # x y org dst | fuel cargo | type a b | tape
_OUT = struct.Struct("<4BBb2xdifd52xi")               # x y org dst done err | fuel cargo rew rew64 | used
_RESET_OUT = struct.Struct("<4B4xdi")
_RESET_IN = struct.Struct("<ii")                      # origin, dest into type, a
_TYPE = 32
_L = dict(x=256, y=272, org=288, dst=304, done=320, err=336, fuel=352, cargo=368, rew=384, rew64=400,
          type=416, a=432, b=448, tape=464)
_SIZE = 512
_I32_MIN, _I32_MAX = -(2 ** 31), 2 ** 31 - 1
_NONE = N.SE_NONE


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
        self._lib = lib
        self.dev = torch.device("cuda", torch.cuda.current_device()) if device is None \
            else torch.device(device)
        if server is None:
            server = os.environ.get("SHIPENV_GPU_SERVER", "1").strip() != "0"
        self.server = bool(server)
        blk = C.c_void_p()
        with torch.cuda.device(self.dev):  # pinned for (mapped into) this GPU
            N.check(lib.se_host_alloc(_SIZE, C.byref(blk)))
        self._blk = blk
        self._mv = memoryview((C.c_uint8 * _SIZE).from_address(blk.value)).cast("B")
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
        L = {k: b + v for k, v in _L.items()}
        self._state = N.SeState(L["x"], L["y"], L["fuel"], L["cargo"], L["org"], L["dst"], L["rew"], L["done"],
                                L["err"], None, None, None, None, L["rew64"])
        N.check(lib.se_bind(self._h, C.byref(self._state)))
        self._base = b
        self._srv = C.c_void_p()
        if self.server:
            N.check(lib.se_server_create(C.byref(self._srv), self._h, b))
        self._sv = self._srv.value

    def set_world(self, water, port_x, port_y, port_fuel, port_cargo):
        """Replace map and ports (a new handle: the map size may change)."""
        self.close()
        self.__init__(water, port_x, port_y, port_fuel, port_cargo, self.dev, self.server)

    def step(self, x, y, fuel, cargo, origin, dest, act_type, a, b, tape):
        """tape: (u_fuel, u_gate, u_type, beta, arrive_dest), NaN / -1 where not drawn."""
        a, b = _clamp32(a), _clamp32(b)
        _IN.pack_into(self._mv, 0, x, y, _NONE if origin is None else origin, _NONE if dest is None else dest,
                      fuel, cargo, act_type, a, b, tape[0], tape[1], tape[2], tape[3], tape[4])
        if self._sv:
            rc = self._lib.se_server_call(self._sv, N.SERVER_STEP)  # answered: results in the block
            if rc:
                N.check(rc)
        else:
            self._launch_step()
        x, y, org, dst, done, err, fuel, cargo, _, r64, used = _OUT.unpack_from(self._mv, 0)
        return StepResult(x, y, fuel, cargo, -1 if org == _NONE else org, -1 if dst == _NONE else dst,
                          r64, bool(done), err, used)

    def reset_to(self, origin, dest):
        _RESET_IN.pack_into(self._mv, _TYPE, origin, dest)
        if self._sv:
            N.check(self._lib.se_server_call(self._sv, N.SERVER_RESET_TO))
        else:
            self._launch_reset_to()
        x, y, org, dst, fuel, cargo = _RESET_OUT.unpack_from(self._mv, 0)
        return StepResult(x, y, fuel, cargo, org, dst, 0.0, False, 0, 0)

    # the launch path: the block's fields through the aligned layout, one launch, one synchronise
    def _copy(self, names, to_aligned):
        mv = self._mv
        src = {"x": 0, "y": 1, "org": 2, "dst": 3, "done": 4, "err": 5, "fuel": 8, "cargo": 16, "rew": 20,
               "rew64": 24, "type": 32, "a": 36, "b": 40}
        size = {"fuel": 8, "rew64": 8, "cargo": 4, "rew": 4, "type": 4, "a": 4, "b": 4}
        for k in names:
            o, n = src[k], size.get(k, 1)
            if to_aligned:
                mv[_L[k]:_L[k] + n] = mv[o:o + n]
            else:
                mv[o:o + n] = mv[_L[k]:_L[k] + n]

    def _launch_step(self):
        mv = self._mv
        self._copy(("x", "y", "org", "dst", "fuel", "cargo", "type", "a", "b"), True)
        mv[_L["tape"]:_L["tape"] + 40] = mv[48:88]
        b_ = self._base
        stream = _raw_stream(self.dev.index)
        N.check(self._lib.se_step_replay(self._h, b_ + _L["type"], b_ + _L["a"], b_ + _L["b"], b_ + _L["tape"],
                                         stream))
        _hip_sync(stream)  # the kernel wrote its results into the pinned memory
        self._copy(("x", "y", "org", "dst", "done", "err", "fuel", "cargo", "rew", "rew64"), False)
        mv[48:88] = mv[_L["tape"]:_L["tape"] + 40]

    def _launch_reset_to(self):
        self._copy(("type", "a"), True)
        b_ = self._base
        stream = _raw_stream(self.dev.index)
        N.check(self._lib.se_reset_to(self._h, None, b_ + _L["type"], b_ + _L["a"], stream))
        _hip_sync(stream)
        self._copy(("x", "y", "org", "dst", "done", "err", "fuel", "cargo", "rew"), False)

    def launches(self):
        """Kernel launches of the stepper wave so far (1 + restarts after idle exits)."""
        n = C.c_uint64()
        N.check(self._lib.se_server_launches(self._srv, C.byref(n)))
        return int(n.value)

    def close(self):
        lib = N.lib()
        if getattr(self, "_srv", None) is not None and self._srv.value:
            lib.se_server_destroy(self._srv)  # ends the wave
            self._srv = C.c_void_p()
            self._sv = None
        if getattr(self, "_h", None) is not None and self._h.value:
            torch.cuda.synchronize(self.dev)
            lib.se_destroy(self._h)
            self._h = C.c_void_p()
        if getattr(self, "_blk", None) is not None and self._blk.value:
            self._mv = None
            lib.se_host_free(self._blk)
            self._blk = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass
