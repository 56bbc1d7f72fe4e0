"""Map setup: the land/sea grid of Environment._initialize_map (shipping/environment.py:45-55).

Host-side, once per environment set (not on the step path). The reference does
    cv2.imread(GRAYSCALE) -> crop rows 50:200, cols 100:300 -> cv2.resize((W, H), INTER_AREA)
    -> cv2.threshold(128, 1, BINARY) -> astype(int)
and indexes the result as np_game[x, y] with x the ROW (:65, :293).
opencv is not part of this image, so the pipeline is restated in C++ in the
library (csrc/mapload.cpp: a baseline/progressive JPEG decoder with libjpeg's
accurate integer IDCT for the Y plane, OpenCV's generic area resampler with
float32 accumulation and round-half-even, threshold ``> 128``). For the
reference's own map this reproduces the committed fixture
(tests/golden/map_water_100x100.bits, sha256 in golden_meta.json); the test-side
checker is mapref.py (Pillow's libjpeg-turbo + a numpy restatement). Agreement with
real cv2 is unpinned (the reference has no map fixture).

``BUILTIN_MAP`` names the derived 100x100 mask bundled with the package, for
machines that do not have the reference's JPEG.
"""
from __future__ import annotations

import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BUILTIN_MAP = "builtin:mapa_mundi_binario"
_BUILTIN_BITS = os.path.join(HERE, "data", "mapa_mundi_binario_100x100.bits")
_REFERENCE_JPEG_NAME = "mapa_mundi_binario.jpg"
_BUNDLED_JPEG = os.path.join(HERE, "data", _REFERENCE_JPEG_NAME)  # the reference's map (data file)


def builtin_water():
    """The reference map after _initialize_map at game_size (100, 100): uint8, 1 = not ground."""
    with open(_BUILTIN_BITS, "rb") as f:
        bits = np.frombuffer(f.read(), np.uint8)
    return np.unpackbits(bits)[: 100 * 100].reshape(100, 100).copy()


_cache = {}


def _native_from_jpeg(data, H, W):
    import ctypes as C

    from . import _native as N

    out = np.zeros(H * W, np.uint8)
    rc = N.lib().se_map_from_jpeg(data, C.c_size_t(len(data)), H, W, out.ctypes.data_as(C.c_void_p))
    if rc:
        raise OSError(N.lib().se_last_error().decode(errors="replace"))
    return out.reshape(H, W)


def load_water(map_path, game_size=(100, 100)):
    """Environment._initialize_map: returns uint8 (H, W), 1 = not ground (WATER), 0 = GROUND.

    The JPEG goes through the library's C++ loader (csrc/mapload.cpp, se_map_from_jpeg:
    libjpeg-exact luma decode, OpenCV's generic INTER_AREA, > 128). A path that does
    not exist but names the reference's map file resolves to the copy bundled with
    the package (the reference's agents open it by bare name, agents/mcts.py:190).
    Decoded masks are cached per (path, mtime, size, game_size): MCTS builds an
    Environment per simulation (agents/mcts.py:199).
    """
    if map_path == BUILTIN_MAP:
        if tuple(game_size) != (100, 100):
            raise ValueError("the builtin map is the 100x100 derivation")
        return builtin_water()
    path = str(map_path)
    if not os.path.exists(path) and os.path.basename(path) == _REFERENCE_JPEG_NAME:
        path = _BUNDLED_JPEG
    if not os.path.exists(path):
        raise FileNotFoundError(f"Cannot read the image at {map_path}")  # environment.py:47
    W, H = game_size  # cv2.resize takes (width, height) (:53)
    st = os.stat(path)
    key = (os.path.abspath(path), st.st_mtime_ns, st.st_size, int(H), int(W))
    hit = _cache.get(key)
    if hit is None:
        with open(path, "rb") as f:
            data = f.read()
        try:
            hit = _native_from_jpeg(data, int(H), int(W))
        except OSError as e:
            raise FileNotFoundError(f"Cannot read the image at {map_path}") from e
        _cache[key] = hit
    return hit.copy()
