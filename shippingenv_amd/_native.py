"""ctypes binding of libshipenv_hip.so (the C-ABI of include/shipenv.h).

There is no fallback: if the gfx950 library is missing or fails to load,
``lib()`` raises ``NativeLibraryError``. The library is built in-tree by
``__graft_entry__.build()`` (or ``python -m shippingenv_amd.build``).
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# SHIPENV_LIB names another build of the same library (an A/B variant under _lib/abl)
LIB_PATH = os.environ.get("SHIPENV_LIB") or os.path.join(HERE, "_lib", "libshipenv_hip.so")
ABI_VERSION = 2  # include/shipenv.h SHIPENV_ABI_VERSION

SE_FLAG_AUTO_RESET = 1
SE_NONE = 255

# per-env error classes (include/shipenv.h SE_ERR_*)
ERR_OK, ERR_OOB, ERR_SAME_PORT, ERR_PORT_RANGE, ERR_NOT_AT_PORT = 0, 1, 2, 3, 4
ERR_AMOUNT, ERR_NO_DEST, ERR_BAD_CATEGORY, ERR_NO_PORTS, ERR_BAD_INDEX = 5, 6, 7, 8, 9
ERR_NEED_DRAW = 10

# se_tape.used bits
USED_FUEL_GATE, USED_LOSS_TYPE, USED_BETA, USED_ARRIVE, USED_MOVED = 1, 2, 4, 8, 16

# se_sample_actions special types, se_rollout statuses
SAMPLE_RAISES, SAMPLE_NO_OTHER_PORT = -1, -2
ROLL_DONE, ROLL_MAX_STEPS, ROLL_RAISED, ROLL_ATTEMPTS, ROLL_BAD_SRC = 0, 1, 2, 3, 4

# se_server_call ops
SERVER_STEP, SERVER_RESET_TO = 1, 2

# every symbol include/shipenv.h declares
EXPORTS = (
    "se_create", "se_set_ports", "se_bind", "se_reset", "se_reset_to", "se_step", "se_step_seq", "se_step_seq_mark",
    "se_step_typed", "se_step_replay", "se_step_agent_replay", "se_observe", "se_valid_mask", "se_gen_actions",
    "se_sample_actions", "se_rollout", "se_qnet_create", "se_qnet_set_weights", "se_policy", "se_policy_f32",
    "se_qnet_repack", "se_policy_record", "se_policy_record_f32",
    "se_qnet_destroy", "se_replay_create", "se_replay_begin", "se_replay_end", "se_replay_end_reset", "se_step_record",
    "se_replay_size",
    "se_replay_sample", "se_replay_destroy", "se_qtrain_create", "se_qtrain_bind", "se_qtrain_pack",
    "se_qtrain_step", "se_qtrain_step_policy", "se_qtrain_step_replay", "se_qtrain_grad_size", "se_qtrain_grad", "se_qtrain_apply",
    "se_qtrain_destroy",
    "se_episode_stats", "se_clear_stats", "se_done_layout", "se_done_list", "se_done_compact",
    "se_get_counters", "se_set_counters",
    "se_map_decode_luma", "se_map_area_threshold", "se_map_from_jpeg",
    "se_host_create", "se_host_set_ports", "se_host_step_replay", "se_host_reset_to", "se_host_destroy",
    "se_host_alloc", "se_host_free", "se_server_create", "se_server_call", "se_server_launches", "se_server_destroy",
    "se_destroy", "se_last_error", "se_abi_version",
)


class NativeLibraryError(RuntimeError):
    pass


class ShipEnvError(RuntimeError):
    """A negative status from the C-ABI (API misuse or a HIP failure)."""


class SeState(C.Structure):
    _fields_ = [(name, C.c_void_p) for name in (
        "x", "y", "fuel", "cargo", "origin", "dest", "reward", "done", "err", "ep_return",
        "ep_start", "done_recs", "done_count", "reward64")]


class SeDoneRec(C.Structure):
    _fields_ = [("env", C.c_int32), ("ep_return", C.c_float), ("ep_len", C.c_int32),
                ("step", C.c_int32)]


_LIB = None


def _declare(lib):
    P, i32, i64, u32, u64 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint32, C.c_uint64
    sig = {
        "se_create": [C.POINTER(P), C.c_int, i64, i64, i32, i32, P, i32, P, P, P, P, u64, u32],
        "se_set_ports": [P, i32, P, P, P, P],
        "se_bind": [P, C.POINTER(SeState)],
        "se_reset": [P, P, P],
        "se_reset_to": [P, P, P, P, P],
        "se_step": [P, P, P],
        "se_step_seq": [P, P, i64, i32, P],
        "se_step_seq_mark": [P, P, i64, i32, P, P, i32],
        "se_step_typed": [P, P, P, P, P],
        "se_step_replay": [P, P, P, P, P, P],
        "se_step_agent_replay": [P, P, P, P],
        "se_observe": [P, P, i64, P],
        "se_valid_mask": [P, P, P],
        "se_gen_actions": [P, P, u32, P],
        "se_sample_actions": [P, P, P, P, u32, P],
        "se_rollout": [P, P, i64, i32, i32, i64, P, P, P, P],
        "se_qnet_create": [C.POINTER(P), P],
        "se_qnet_set_weights": [P, P, P, P, P, P, P, P],
        "se_policy": [P, P, C.c_double, u32, P, i64, P],
        "se_policy_f32": [P, P, C.c_double, u32, P, i64, P],
        "se_qnet_repack": [P, P, P],
        "se_policy_record": [P, P, P, C.c_double, u32, P],
        "se_policy_record_f32": [P, P, P, C.c_double, u32, P],
        "se_qnet_destroy": [P],
        "se_replay_create": [P, P, i64],
        "se_replay_begin": [P, P, P],
        "se_replay_end": [P, P, C.c_int32, P],
        "se_replay_end_reset": [P, P, C.c_int32, P],
        "se_step_record": [P, P, P, C.c_int32, P],
        "se_replay_size": [P, P, P],
        "se_replay_sample": [P, i64, P, u32, P, P, P, P, P, P, P],
        "se_replay_destroy": [P],
        "se_qtrain_create": [P, P, i64],
        "se_qtrain_bind": [P, P, P, P, P, P],
        "se_qtrain_pack": [P, C.c_int32, P],
        "se_qtrain_step": [P, i64, P, P, P, P, P, P] + [C.c_float] * 5 + [P, P, P],
        "se_qtrain_step_policy": [P, P, i64, P, P, P, P, P, P] + [C.c_float] * 5 + [P, P, P],
        "se_qtrain_step_replay": [P, P, P, i64] + [C.c_float] * 5 + [P, i64, P, P],
        "se_qtrain_grad_size": [P],
        "se_qtrain_grad": [P, i64, P, P, P, P, P, P, C.c_float, P, P],
        "se_qtrain_apply": [P, P, P] + [C.c_float] * 4 + [P, P, P],
        "se_qtrain_destroy": [P],
        "se_episode_stats": [P, P, P],
        "se_clear_stats": [P, P],
        "se_done_layout": [P, C.POINTER(i64), C.POINTER(i32)],
        "se_done_list": [P, C.POINTER(i64), C.POINTER(i64)],
        "se_done_compact": [P, P, P, P],
        "se_get_counters": [P, C.POINTER(u64), C.POINTER(u64)],
        "se_set_counters": [P, u64, u64],
        "se_map_decode_luma": [C.c_char_p, C.c_size_t, P, C.c_size_t, C.POINTER(i32), C.POINTER(i32)],
        "se_map_area_threshold": [P, i32, i32, i32, i32, i32, i32, i32, i32, C.c_uint8, P, P],
        "se_map_from_jpeg": [C.c_char_p, C.c_size_t, i32, i32, P],
        "se_host_create": [C.POINTER(P), i32, i32, P, i32, P, P, P, P],
        "se_host_set_ports": [P, i32, P, P, P, P],
        "se_host_step_replay": [P, i64, P, P, P, P, P],
        "se_host_reset_to": [P, i64, P, P, P, P],
        "se_host_destroy": [P],
        "se_host_alloc": [C.c_size_t, C.POINTER(P)],
        "se_host_free": [P],
        "se_server_create": [C.POINTER(P), P, P],
        "se_server_call": [P, i32],
        "se_server_launches": [P, C.POINTER(C.c_uint64)],
        "se_server_destroy": [P],
        "se_destroy": [P],
        "se_last_error": [],
        "se_abi_version": [],
    }
    for name, args in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = C.c_int
    lib.se_last_error.restype = C.c_char_p
    lib.se_qtrain_grad_size.restype = i64


def lib():
    """Load the gfx950 library (once). Raises NativeLibraryError if it is unusable."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (hipcc --offload-arch=gfx950). There is no CPU fallback.")
    # torch's ROCm runtime loads first. It ships its own HIP and an HSA runtime with the
    # soname libhsa-runtime64.so.1, the same soname as /opt/rocm's, which this library
    # needs: whichever is loaded first serves both HIP runtimes in the process. Loaded
    # before torch (shipping.Environment(<jpeg>) decodes the map through this library
    # before anything touches the GPU, as the reference's MCTS agent does), the
    # library's HIP later found no device once torch's runtime had initialised
    # (tests/test_compat_gpu.py::test_library_loaded_before_torch).
    import torch  # noqa: F401
    if os.environ.get("SHIPENV_LIB"):  # an A/B variant replaces the product library: say so
        import sys
        print(f"shippingenv_amd: SHIPENV_LIB overrides the library: {LIB_PATH}", file=sys.stderr, flush=True)
    try:
        handle = C.CDLL(LIB_PATH)
    except OSError as e:
        raise NativeLibraryError(f"cannot load {LIB_PATH}: {e}") from e
    missing = [s for s in EXPORTS if not hasattr(handle, s)]
    if missing:
        raise NativeLibraryError(f"{LIB_PATH} lacks symbols {missing}")
    _declare(handle)
    if handle.se_abi_version() != ABI_VERSION:
        raise NativeLibraryError("ABI version mismatch; rebuild the library")
    _LIB = handle
    return _LIB


def check(rc):
    if rc != 0:
        msg = lib().se_last_error().decode(errors="replace")
        raise ShipEnvError(f"shipenv status {rc}: {msg}")
    return rc
