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
