"""CPU restatement of Environment._initialize_map (test infrastructure only).

The reference (/root/reference/shipping/environment.py:45-55) does
    cv2.imread(path, IMREAD_GRAYSCALE) -> crop [50:200, 100:300]
    -> cv2.resize((W, H), INTER_AREA) -> cv2.threshold(128, 1, BINARY)
opencv is not installed here, so this checker decodes with Pillow's
libjpeg-turbo (draft "L" = the Y component, accurate integer IDCT: what
IMREAD_GRAYSCALE returns for a JPEG) and restates OpenCV's generic area
resampler: computeResizeAreaTab weights (f64 positions, f32 weights) and
ResizeArea_Invoker's float32 accumulation (per source row, x-terms in ascending
source column; then rows weighted in ascending source row), rounded half to even.
Pinned by the committed mask fixture (tests/golden/map_water_100x100.bits,
sha256 49253a2c... = the survey's probe); agreement with real cv2 is unpinned
(the reference has no map test). The product path is
shippingenv_amd/csrc/mapload.cpp; only tests/ import this module.
"""
from __future__ import annotations

import io
import math

import numpy as np


def decode_luma(data: bytes) -> np.ndarray:
    from PIL import Image

    im = Image.open(io.BytesIO(data))
    im.draft("L", im.size)
    return np.array(im.convert("L"), np.uint8)


def area_weights(ssize, dsize):
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
    """cv2.resize(src, (width, height), interpolation=INTER_AREA), uint8 gray, generic scale."""
    src = np.asarray(src, np.uint8)
    sh, sw = src.shape
    wx = area_weights(sw, width)
    wy = area_weights(sh, height)
    f32 = np.float32
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


def initialize_map(data: bytes, game_size=(100, 100)) -> np.ndarray:
    """uint8 (H, W): 1 where the resized luma is > 128 (not GROUND), 0 = GROUND."""
    gray = decode_luma(data)
    crop = gray[50:200, 100:300]
    W, H = game_size
    return (resize_area(crop, W, H) > 128).astype(np.uint8)
