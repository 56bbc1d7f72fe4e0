"""The drop-in shipping.Environment on the MI355X (HIP step kernel through the
C-ABI, SHIPENV_STEPPER=gpu) against the reference's own seeded traces: identical
results, Python types, exceptions and global `random` stream; and its default host
stepper (the same per-env code compiled for the host) against the kernel, bit for bit."""
import time

import pytest

from compat_replay import load_script, replay

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _device_backend(monkeypatch):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from shippingenv_amd.shipping import environment

    environment._set_stepper_factory(None)
    monkeypatch.setenv("SHIPENV_STEPPER", "gpu")  # the kernel: DeviceStepper


@pytest.mark.parametrize("seed", range(6))
def test_seeded_trace_matches_reference_on_gpu(seed):
    assert replay(load_script(seed)) > 600


def test_steps_run_through_the_hip_library():
    import ctypes

    from shippingenv_amd import _native
    from shippingenv_amd.maps import BUILTIN_MAP
    from shippingenv_amd.shipping import Environment
    from shippingenv_amd.shipping._device import DeviceStepper

    env = Environment(BUILTIN_MAP)
    for p in ([41, 40], [60, 22], [78, 29]):
        env.add_port(p)
    env.reset()
    assert isinstance(env._stepper, DeviceStepper)
    assert isinstance(_native.lib(), ctypes.CDLL)
    t0 = time.perf_counter()
    for _ in range(200):
        try:
            env.step([1, (0, 1)])
        except ValueError:
            env.step([1, (0, -1)])
    dt = (time.perf_counter() - t0) / 200
    print(f"compat step: {dt * 1e6:.1f} us")
    assert dt < 5e-3


def test_library_loaded_before_torch():
    """The reference's MCTS agent imports shipping but not torch (agents/mcts.py:3-10)
    and builds Environment("mapa_mundi_binario.jpg"), whose map decode loads the
    library before torch: the steps must still run on the GPU (a fresh interpreter)."""
    import os
    import subprocess
    import sys

    from conftest import ROOT

    code = (
        "import sys; from shippingenv_amd.shipping import Environment\n"
        "env = Environment('mapa_mundi_binario.jpg')\n"
        "env.add_port([41, 40]); env.add_port([60, 22])\n"
        "env.reset()\n"
        "from shippingenv_amd.shipping._device import DeviceStepper\n"
        "assert isinstance(env._stepper, DeviceStepper)\n"
        "env.step([1, (0, 1)]) if env.np_game[41, 41] != 0 else env.step([1, (0, -1)])\n"
        "print('ok')\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, PYTHONPATH=ROOT, SHIPENV_STEPPER="gpu"))
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


# ------------------------------------------------------------------ host stepper vs kernel
def _kernel_replay(z, sel, water, with_ports):
    import numpy as np

    from shippingenv_amd.vec import TAPE_DTYPE, VecEnv

    sl = slice(None) if with_ports else slice(0, 0)
    ports = [[int(a), int(b)] for a, b in zip(z["port_x"][sl], z["port_y"][sl])]
    env = VecEnv(len(sel), water=water, ports=ports, port_fuel=z["port_fuel"][sl], port_cargo=z["port_cargo"][sl])
    for f in ("x", "y", "fuel", "cargo", "origin", "dest"):
        v = z["pre_" + f][sel]
        if f in ("origin", "dest"):
            v = np.where(v < 0, 255, v)
        t = getattr(env, f)
        t.copy_(torch.from_numpy(np.ascontiguousarray(v).astype(t.cpu().numpy().dtype)))
    tape = np.zeros(len(sel), TAPE_DTYPE)
    for f in ("u_fuel", "u_gate", "u_type", "beta", "arrive_dest"):
        tape[f] = z[f][sel]
    env.step_replay(z["act_type"][sel], z["act_a"][sel], z["act_b"][sel], tape)
    torch.cuda.synchronize()
    out = {f: getattr(env, f).cpu().numpy() for f in ("x", "y", "fuel", "cargo", "origin", "dest", "reward",
                                                        "done", "err")}
    env.close()
    return out


def _golden():
    from conftest import golden_files

    return golden_files()


@pytest.mark.parametrize("path", _golden(), ids=lambda p: p.rsplit("/", 1)[-1])
def test_host_stepper_equals_kernel_on_golden_records(path, water):
    """se_host_step_replay (host build of replay_env) and se_step_replay (the kernel) on
    every golden record: every field bit for bit."""
    import numpy as np

    from conftest import load_golden
    from test_host_step import host_replay

    z = load_golden(path)
    n = 0
    for kind, with_ports in ((0, True), (2, False)):
        sel = np.nonzero(z["kind"] == kind)[0]
        if not len(sel):
            continue
        k = _kernel_replay(z, sel, water, with_ports)
        h = host_replay(z, sel, water, with_ports)
        for f, v in k.items():
            hv = h[f]
            if f == "fuel":
                np.testing.assert_array_equal(hv.view(np.int64), v.view(np.int64), err_msg=f)
            elif f == "reward":
                np.testing.assert_array_equal(hv.view(np.int32), v.view(np.int32), err_msg=f)
            else:
                np.testing.assert_array_equal(hv.astype(np.int64), v.astype(np.int64), err_msg=f)
        n += len(sel)
    assert n > 1000


@pytest.mark.parametrize("seed", range(6))
def test_host_and_gpu_steppers_give_the_same_trace(monkeypatch, seed):
    """The drop-in on either stepper reproduces the reference's seeded trace (the replay
    checks every step against it), so the two steppers agree step for step."""
    assert replay(load_script(seed)) > 600  # SHIPENV_STEPPER=gpu (fixture)
    monkeypatch.setenv("SHIPENV_STEPPER", "host")
    assert replay(load_script(seed)) > 600


def test_default_stepper_is_host_and_gpu_is_selectable(monkeypatch):
    from shippingenv_amd.maps import BUILTIN_MAP
    from shippingenv_amd.shipping import Environment
    from shippingenv_amd.shipping._device import DeviceStepper
    from shippingenv_amd.shipping._host import HostStepper

    for kind, cls in (("gpu", DeviceStepper), ("host", HostStepper)):
        monkeypatch.setenv("SHIPENV_STEPPER", kind)
        env = Environment(BUILTIN_MAP)
        env.add_port([41, 40])
        env.add_port([60, 22])
        env.reset()
        assert isinstance(env._stepper, cls)
    monkeypatch.delenv("SHIPENV_STEPPER")
    env = Environment(BUILTIN_MAP)
    env.add_port([41, 40])
    env.add_port([60, 22])
    env.reset()
    assert isinstance(env._stepper, HostStepper)


@pytest.mark.parametrize("seed", range(2))
def test_seeded_trace_on_the_launch_stepper(monkeypatch, seed):
    """SHIPENV_GPU_SERVER=0: one se_step_replay launch and one synchronise per step instead of
    the resident stepper wave; the same reference traces."""
    monkeypatch.setenv("SHIPENV_GPU_SERVER", "0")
    assert replay(load_script(seed)) > 600


def test_stepper_wave_restarts_after_idle(monkeypatch):
    """The resident stepper wave (csrc/server.h) ends after 20 ms without a command and the
    next step launches it again: pauses of 50 ms inside a run give the same results as the
    host stepper, step for step, and the wave was launched once per pause."""
    import random

    from shippingenv_amd.maps import BUILTIN_MAP
    from shippingenv_amd.shipping import Environment
    from shippingenv_amd.shipping._device import DeviceStepper

    def run(kind, pause):
        monkeypatch.setenv("SHIPENV_STEPPER", kind)
        random.seed(7)
        env = Environment(BUILTIN_MAP)
        for p in ([41, 40], [60, 22], [78, 29]):
            env.add_port(p)
        env.reset()
        out = []
        for k in range(90):
            if pause and k % 30 == 15:
                time.sleep(0.05)
            try:
                out.append(repr(env.step([1, (0, 1) if k % 3 else (1, 0)])))
            except Exception as e:  # noqa: BLE001 - the reference's exceptions are part of the trace
                out.append(f"{type(e).__name__}: {e}")
        launches = env._stepper.launches() if isinstance(env._stepper, DeviceStepper) else None
        return out, launches

    host, _ = run("host", False)
    gpu, launches = run("gpu", True)
    assert gpu == host
    assert launches >= 4, launches


def test_stepper_wave_refuses_misuse():
    """se_server_create checks its block (pinned host memory from se_host_alloc, 64-byte
    aligned) and takes a one-env handle only; se_server_call takes the two ops only; destroy
    of NULL is a no-op. A refused block leaves no HIP error behind: the next step launches."""
    import ctypes as C

    import numpy as np

    from shippingenv_amd import _native as N
    from shippingenv_amd.maps import BUILTIN_MAP, builtin_water
    from shippingenv_amd.shipping import Environment

    lib = N.lib()
    water = np.ascontiguousarray(builtin_water(), np.uint8)
    H, W = water.shape
    px, py, pf, pc = (np.ascontiguousarray(v, np.int32) for v in ([41, 60], [40, 22], [100, 100], [10, 10]))

    def env_of(n):
        h = C.c_void_p()
        N.check(lib.se_create(C.byref(h), torch.cuda.current_device(), n, 0, H, W,
                              water.ctypes.data_as(C.c_void_p), 2, px.ctypes.data_as(C.c_void_p),
                              py.ctypes.data_as(C.c_void_p), pf.ctypes.data_as(C.c_void_p),
                              pc.ctypes.data_as(C.c_void_p), 0, 0))
        return h

    blk = C.c_void_p()
    N.check(lib.se_host_alloc(256, C.byref(blk)))
    env1, env2 = env_of(1), env_of(2)
    srv = C.c_void_p()
    try:
        pageable = np.zeros(512, np.uint8)
        aligned = pageable.ctypes.data + (-pageable.ctypes.data) % 64
        assert lib.se_server_create(C.byref(srv), env1, aligned) < 0 and not srv.value
        assert lib.se_server_create(C.byref(srv), env1, blk.value + 16) < 0  # not 64-byte aligned
        assert lib.se_server_create(C.byref(srv), env2, blk.value) < 0  # two envs
        assert lib.se_server_create(C.byref(srv), env1, None) < 0
        assert lib.se_server_create(C.byref(srv), None, blk.value) < 0
        N.check(lib.se_server_create(C.byref(srv), env1, blk.value))
        assert lib.se_server_call(srv, 0) < 0 and lib.se_server_call(srv, 3) < 0
        assert lib.se_server_call(None, N.SERVER_STEP) < 0
        n = C.c_uint64()
        N.check(lib.se_server_launches(srv, C.byref(n)))
        assert n.value == 0  # the wave starts with the first step
        N.check(lib.se_server_destroy(srv))
        srv = C.c_void_p()
        assert lib.se_server_destroy(None) == 0
    finally:
        if srv.value:
            lib.se_server_destroy(srv)
        lib.se_destroy(env1)
        lib.se_destroy(env2)
        lib.se_host_free(blk)
    env = Environment(BUILTIN_MAP)  # same thread, after the refused pageable block
    env.add_port([41, 40])
    env.add_port([60, 22])
    env.reset()
    env.step([1, (0, 1)]) if env.np_game[41, 41] != 0 else env.step([1, (0, -1)])
    assert env._stepper.launches() >= 1
