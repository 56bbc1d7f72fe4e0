"""The C++ map loader (csrc/mapload.cpp, include/shipenv.h se_map_*) against the
checkers: libjpeg-turbo's luma planes (tests/golden/jpeg, made by
tests/golden/make_jpeg_golden.py), oracle/mapref.py's restatement of OpenCV's
INTER_AREA, and the committed map fixture (Environment._initialize_map,
shipping/environment.py:45-55). Host code only: runs without a GPU."""
import ctypes as C
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden_water
from oracle import mapref
from shippingenv_amd import _native as N
from shippingenv_amd import maps

JPEG_DIR = os.path.join(GOLDEN, "jpeg")
META = json.load(open(os.path.join(JPEG_DIR, "jpeg_meta.json")))
REF_MAP = os.path.join(os.path.dirname(maps.__file__), "data", "mapa_mundi_binario.jpg")


def decode(data):
    lib = N.lib()
    h, w = C.c_int32(), C.c_int32()
    N.check(lib.se_map_decode_luma(data, len(data), None, 0, C.byref(h), C.byref(w)))
    out = np.zeros(h.value * w.value, np.uint8)
    N.check(lib.se_map_decode_luma(data, len(data), out.ctypes.data_as(C.c_void_p), out.size,
                                   C.byref(h), C.byref(w)))
    return out.reshape(h.value, w.value)


def area(gray, r0, r1, c0, c1, H, W, thr=128):
    lib = N.lib()
    g = np.ascontiguousarray(gray, np.uint8)
    res = np.zeros(H * W, np.uint8)
    mask = np.zeros(H * W, np.uint8)
    N.check(lib.se_map_area_threshold(g.ctypes.data_as(C.c_void_p), g.shape[0], g.shape[1], r0, r1,
                                      c0, c1, H, W, thr, res.ctypes.data_as(C.c_void_p),
                                      mask.ctypes.data_as(C.c_void_p)))
    return res.reshape(H, W), mask.reshape(H, W)


@pytest.mark.parametrize("name", META["cases"])
def test_luma_matches_libjpeg(name):
    """Baseline / progressive, 4:2:0 / 4:2:2 / 4:4:4 / gray, odd sizes, restarts: bit-exact."""
    with open(os.path.join(JPEG_DIR, f"{name}.jpg"), "rb") as f:
        data = f.read()
    want = np.load(os.path.join(JPEG_DIR, "jpeg_luma.npz"))[name]
    got = decode(data)
    assert got.shape == want.shape
    assert np.array_equal(got, want)


def test_reference_map_luma_and_mask():
    """The reference's own map (progressive 4:2:0 with successive approximation)."""
    with open(REF_MAP, "rb") as f:
        data = f.read()
    luma = decode(data)
    assert list(luma.shape) == META["reference_map_luma"]["shape"]
    assert hashlib.sha256(luma.tobytes()).hexdigest() == META["reference_map_luma"]["sha256"]
    water = np.zeros(100 * 100, np.uint8)
    N.check(N.lib().se_map_from_jpeg(data, len(data), 100, 100, water.ctypes.data_as(C.c_void_p)))
    meta = json.load(open(os.path.join(GOLDEN, "golden_meta.json")))["map"]
    assert hashlib.sha256(water.tobytes()).hexdigest() == meta["sha256_u8_rowmajor"]
    assert np.array_equal(water.reshape(100, 100), golden_water())


def test_reference_map_vs_oracle_pipeline():
    with open(REF_MAP, "rb") as f:
        data = f.read()
    assert np.array_equal(maps.load_water(REF_MAP), mapref.initialize_map(data))


@pytest.mark.parametrize("shape,crop,size", [
    ((355, 533), (50, 200, 100, 300), (100, 100)),
    ((355, 533), (50, 200, 100, 300), (64, 37)),
    ((120, 90), (0, 120, 0, 90), (17, 13)),
    ((40, 40), (3, 40, 5, 33), (37, 28)),
    ((64, 64), (0, 64, 0, 64), (32, 16)),  # integer scales on the generic path
])
def test_area_resize_vs_oracle(shape, crop, size):
    rng = np.random.default_rng(sum(shape) + sum(size))
    gray = rng.integers(0, 256, size=shape, dtype=np.uint8)
    gray[::7] = 128  # plateaus at the threshold
    r0, r1, c0, c1 = crop
    H, W = size
    res, mask = area(gray, r0, r1, c0, c1, H, W)
    want = mapref.resize_area(gray[r0:r1, c0:c1], W, H)
    assert np.array_equal(res, want)
    assert np.array_equal(mask, (want > 128).astype(np.uint8))


def test_load_water_paths(tmp_path):
    w = maps.load_water(REF_MAP)
    assert np.array_equal(w, maps.builtin_water())
    # the reference's agents open the map by bare name (agents/mcts.py:190)
    assert np.array_equal(maps.load_water("mapa_mundi_binario.jpg"), w)
    with pytest.raises(FileNotFoundError, match="Cannot read the image at"):
        maps.load_water(str(tmp_path / "missing.jpg"))
    bad = tmp_path / "bad.jpg"
    bad.write_bytes(b"\xff\xd8\xff\xc4\x00\x03\x00")
    with pytest.raises(FileNotFoundError, match="Cannot read the image at"):
        maps.load_water(str(bad))


@pytest.mark.parametrize("cut", [2, 100, 1000, 5000])
def test_truncated_or_corrupt_files_fail_cleanly(cut):
    with open(REF_MAP, "rb") as f:
        data = f.read()
    lib = N.lib()
    h, w = C.c_int32(), C.c_int32()
    # truncated: an error status (libjpeg would warn and pad with zeros; the loader refuses)
    rc = lib.se_map_decode_luma(data[:cut], cut, None, 0, C.byref(h), C.byref(w))
    assert rc in (0, -1)  # SE_OK / SE_EINVAL
    # garbage after the SOI marker never crashes
    rng = np.random.default_rng(cut)
    junk = b"\xff\xd8" + rng.integers(0, 256, size=cut, dtype=np.uint8).tobytes()
    lib.se_map_decode_luma(junk, len(junk), None, 0, C.byref(h), C.byref(w))
