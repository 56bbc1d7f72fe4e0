"""Minimal stand-in for the three OpenCV calls the reference's map loader makes.

Fixture-generation only (tests/golden/make_golden.py); never imported by the
product. opencv-python is pinned by the reference (requirements.txt:8) but is not
installed in this image and nothing may be fetched, so the three calls used at
shipping/environment.py:46,53,54 are restated:

* imread(path, IMREAD_GRAYSCALE): PIL JPEG decode in libjpeg's JCS_GRAYSCALE
  output mode (``draft('L')`` = the Y channel), the same output mode OpenCV's
  JPEG decoder requests for a grayscale read of a colour JPEG.
* resize(src, (W, H), INTER_AREA): OpenCV's generic area resampler (the path
  taken when either scale is non-integer): computeResizeAreaTab weights as
  float32, row accumulation in float32, saturate_cast<uchar> = round-half-even.
* threshold(src, t, maxval, THRESH_BINARY): src > t ? maxval : 0.

GUI calls are no-ops. Parity of this stub against real cv2 is UNPINNED (the
reference has no tests and no fixture of its map); the committed mask fixture
(sha256 in tests/golden/README.md) is the contract.
"""
import math

import numpy as np
from PIL import Image

IMREAD_GRAYSCALE = 0
INTER_AREA = 3
THRESH_BINARY = 0
FONT_HERSHEY_SIMPLEX = 0
LINE_AA = 16


def imread(path, flags=1):
    try:
        im = Image.open(path)
    except (FileNotFoundError, OSError):
        return None
    im.draft("L", im.size)
    im = im.convert("L")
    return np.array(im, dtype=np.uint8)


def _area_tab(ssize, dsize, scale):
    tab = []
    for dx in range(dsize):
        fsx1 = dx * scale
        fsx2 = fsx1 + scale
        cell = min(scale, ssize - fsx1)
        sx1, sx2 = math.ceil(fsx1), math.floor(fsx2)
        sx2 = min(sx2, ssize - 1)
        sx1 = min(sx1, sx2)
        if sx1 - fsx1 > 1e-3:
            tab.append((dx, sx1 - 1, np.float32((sx1 - fsx1) / cell)))
        for sx in range(sx1, sx2):
            tab.append((dx, sx, np.float32(1.0 / cell)))
        if fsx2 - sx2 > 1e-3:
            tab.append((dx, sx2, np.float32(min(min(fsx2 - sx2, 1.0), cell) / cell)))
    return tab


def resize(src, dsize, interpolation=INTER_AREA):
    assert interpolation == INTER_AREA and src.ndim == 2 and src.dtype == np.uint8
    W, H = dsize
    sh, sw = src.shape
    xtab = _area_tab(sw, W, sw / W)
    ytab = _area_tab(sh, H, sh / H)
    dst = np.zeros((H, W), np.uint8)
    f32 = np.float32

    def flush(row, acc):
        dst[row] = np.clip(np.rint(acc), 0, 255).astype(np.uint8)

    acc = np.zeros(W, f32)
    prev_dy = ytab[0][0]
    for dy, sy, beta in ytab:
        buf = np.zeros(W, f32)
        srow = src[sy].astype(f32)
        for dx, sx, alpha in xtab:
            buf[dx] = f32(buf[dx] + f32(srow[sx] * alpha))
        if dy != prev_dy:
            flush(prev_dy, acc)
            acc = (beta * buf).astype(f32)
            prev_dy = dy
        else:
            acc = (acc + (beta * buf).astype(f32)).astype(f32)
    flush(prev_dy, acc)
    return dst


def threshold(src, thresh, maxval, type_=THRESH_BINARY):
    out = np.where(src > thresh, maxval, 0).astype(src.dtype)
    return thresh, out


def imshow(*a, **k):
    pass


def waitKey(*a, **k):
    return -1


def destroyAllWindows(*a, **k):
    pass


def putText(*a, **k):
    pass
