import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libshipenv_hip.so)")


def golden_files(prefix=""):
    return sorted(glob.glob(os.path.join(GOLDEN, f"{prefix}*_seed*.npz")))


def load_golden(path):
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def golden_water():
    with open(os.path.join(GOLDEN, "map_water_100x100.bits"), "rb") as f:
        bits = np.frombuffer(f.read(), np.uint8)
    return np.unpackbits(bits)[:10000].reshape(100, 100).copy()


@pytest.fixture(scope="session")
def water():
    return golden_water()


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle as O

    O.build()
    return O
