"""The drop-in shipping.Environment on the MI355X (HIP step kernel through the
C-ABI) against the reference's own seeded traces: identical results, Python
types, exceptions and global `random` stream."""
import time

import pytest

from compat_replay import load_script, replay

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _device_backend():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from shippingenv_amd.shipping import environment

    environment._set_stepper_factory(None)  # the product path: DeviceStepper


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
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]
