"""Map setup: the land/sea grid of Environment._initialize_map (shipping/environment.py:45-55).

Host-side, once per environment set (not on the step path). The reference does
    cv2.imread(GRAYSCALE) -> crop rows 50:200, cols 100:300 -> cv2.resize((W, H), INTER_AREA)
    -> cv2.threshold(128, 1, BINARY) -> astype(int)
and indexes the result as np_game[x, y] with x the ROW (:65, :293).
opencv is not part of this image, so the pipeline is restated here:
JPEG -> libjpeg grayscale (Y) through PIL, OpenCV's generic area resampler
(computeResizeAreaTab weights in float32, float32 accumulation, round-half-even),
threshold ``> 128``. For the reference's own map this reproduces the committed
fixture (tests/golden/map_water_100x100.bits, sha256 in golden_meta.json);
agreement with real cv2 is unpinned (the reference has no map fixture).

``BUILTIN_MAP`` names the derived 100x100 mask bundled with the package, for
machines that do not have the reference's JPEG.
"""
from __future__ import annotations

import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BUILTIN_MAP = "builtin:mapa_mundi_binario"
_BUILTIN_BITS = os.path.join(HERE, "data", "mapa_mundi_binario_100x100.bits")
_REFERENCE_JPEG_NAME = "mapa_mundi_binario.jpg"


def builtin_water():
    """The reference map after _initialize_map at game_size (100, 100): uint8, 1 = not ground."""
    with open(_BUILTIN_BITS, "rb") as f:
        bits = np.frombuffer(f.read(), np.uint8)
    return np.unpackbits(bits)[: 100 * 100].reshape(100, 100).copy()


def _area_weights(ssize, dsize):
    """OpenCV computeResizeAreaTab as a dense (dsize, ssize) float32 matrix."""
    scale = ssize / dsize
    m = np.zeros((dsize, ssize), np.float32)
    for dx in range(dsize):
        fsx1 = dx * scale
        fsx2 = fsx1 + scale
        cell = min(scale, ssize - fsx1)
        sx1, sx2 = math.ceil(fsx1), math.floor(fsx2)
        sx2 = min(sx2, ssize - 1)
        sx1 = min(sx1, sx2)
        if sx1 - fsx1 > 1e-3:
            m[dx, sx1 - 1] = np.float32((sx1 - fsx1) / cell)
        for sx in range(sx1, sx2):
            m[dx, sx] = np.float32(1.0 / cell)
        if fsx2 - sx2 > 1e-3:
            m[dx, sx2] = np.float32(min(min(fsx2 - sx2, 1.0), cell) / cell)
    return m


def resize_area(src, width, height):
    """cv2.resize(src, (width, height), interpolation=INTER_AREA) for uint8 gray images
    on the generic (non-integer scale) path, accumulation order as OpenCV's
    ResizeArea_Invoker: per source row, x-weights summed left to right in float32,
    then rows weighted and summed top to bottom in float32."""
    src = np.asarray(src, np.uint8)
    sh, sw = src.shape
    wx = _area_weights(sw, width)
    wy = _area_weights(sh, height)
    f32 = np.float32
    # row pass: buf[sy, dx] = sum_sx src[sy, sx] * wx[dx, sx], in ascending sx
    buf = np.zeros((sh, width), f32)
    srcf = src.astype(f32)
    for sx in range(sw):
        col = wx[:, sx]
        nz = np.nonzero(col)[0]
        if len(nz):
            buf[:, nz] = (buf[:, nz] + (srcf[:, sx:sx + 1] * col[nz][None, :]).astype(f32)).astype(f32)
    out = np.zeros((height, width), np.uint8)
    for dy in range(height):
        acc = None
        for sy in np.nonzero(wy[dy])[0]:
            term = (wy[dy, sy] * buf[sy]).astype(f32)
            acc = term if acc is None else (acc + term).astype(f32)
        out[dy] = np.clip(np.rint(acc), 0, 255).astype(np.uint8)
    return out


def load_water(map_path, game_size=(100, 100)):
    """Environment._initialize_map: returns uint8 (H, W), 1 = not ground (WATER), 0 = GROUND."""
    if map_path == BUILTIN_MAP:
        if tuple(game_size) != (100, 100):
            raise ValueError("the builtin map is the 100x100 derivation")
        return builtin_water()
    if not os.path.exists(map_path):
        raise FileNotFoundError(f"Cannot read the image at {map_path}")  # environment.py:47
    from PIL import Image

    try:
        im = Image.open(map_path)
        im.draft("L", im.size)
        gray = np.array(im.convert("L"), np.uint8)
    except OSError as e:
        raise FileNotFoundError(f"Cannot read the image at {map_path}") from e
    crop = gray[50:200, 100:300]  # environment.py:49-52
    W, H = game_size  # cv2.resize takes (width, height) (:53)
    small = resize_area(crop, W, H)
    return (small > 128).astype(np.uint8)  # :54
