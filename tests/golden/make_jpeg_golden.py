"""Generate the JPEG decoder fixtures (tests/test_mapload.py).

    python tests/golden/make_jpeg_golden.py

Writes tests/golden/jpeg/*.jpg (small synthetic images, encoded by Pillow's
libjpeg-turbo in several processes: baseline / progressive, 4:2:0 / 4:2:2 /
4:4:4 / grayscale, odd sizes, restart intervals) and jpeg_luma.npz with, for
each file, the luma plane libjpeg-turbo decodes (Pillow, draft mode "L": the Y
component, accurate integer IDCT) — the output cv2.imread(IMREAD_GRAYSCALE)
gives for a JPEG. Also records the sha256 of the reference map's luma plane
(/root/reference/mapa_mundi_binario.jpg, decoded the same way) in
jpeg_meta.json. Test infrastructure: the product loader is
shippingenv_amd/csrc/mapload.cpp.
"""
import hashlib
import io
import json
import os

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "jpeg")
REF_MAP = "/root/reference/mapa_mundi_binario.jpg"


def decode_luma(data):
    im = Image.open(io.BytesIO(data))
    im.draft("L", im.size)
    return np.array(im.convert("L"), np.uint8)


def synthetic(h, w, seed):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    base = (128 + 90 * np.sin(x / 5.0) * np.cos(y / 7.0)).astype(np.int64)
    edges = ((x // 9 + y // 6) % 2) * 60
    noise = rng.integers(-25, 26, size=(h, w))
    r = np.clip(base + edges + noise, 0, 255)
    g = np.clip(255 - base + noise, 0, 255)
    b = np.clip((base * 3 + edges) % 256, 0, 255)
    return np.stack([r, g, b], -1).astype(np.uint8)


CASES = [
    # name, (h, w), mode, save kwargs
    ("base420", (45, 67), "RGB", dict(quality=85, subsampling=2)),
    ("base444", (33, 50), "RGB", dict(quality=92, subsampling=0)),
    ("base422", (40, 41), "RGB", dict(quality=75, subsampling=1)),
    ("gray", (37, 23), "L", dict(quality=80)),
    ("prog420", (45, 67), "RGB", dict(quality=85, subsampling=2, progressive=True)),
    ("prog444", (29, 31), "RGB", dict(quality=60, subsampling=0, progressive=True)),
    ("proggray", (50, 50), "L", dict(quality=90, progressive=True)),
    ("base_rst", (48, 64), "RGB", dict(quality=85, restart_marker_blocks=3)),
    ("prog_rst", (61, 77), "RGB", dict(quality=70, progressive=True, restart_marker_rows=1)),
    ("q100", (16, 16), "RGB", dict(quality=100, subsampling=0)),
    ("q5", (70, 90), "RGB", dict(quality=5)),
]


def main():
    os.makedirs(OUT, exist_ok=True)
    luma = {}
    for i, (name, (h, w), mode, kw) in enumerate(CASES):
        rgb = synthetic(h, w, seed=100 + i)
        im = Image.fromarray(rgb)
        if mode == "L":
            im = im.convert("L")
        buf = io.BytesIO()
        im.save(buf, "JPEG", **kw)
        data = buf.getvalue()
        with open(os.path.join(OUT, f"{name}.jpg"), "wb") as f:
            f.write(data)
        luma[name] = decode_luma(data)
    np.savez_compressed(os.path.join(OUT, "jpeg_luma.npz"), **luma)
    meta = {"cases": [c[0] for c in CASES], "decoder": "Pillow (libjpeg-turbo), draft('L')"}
    if os.path.exists(REF_MAP):
        with open(REF_MAP, "rb") as f:
            ref = decode_luma(f.read())
        meta["reference_map_luma"] = {"shape": list(ref.shape),
                                      "sha256": hashlib.sha256(ref.tobytes()).hexdigest()}
    with open(os.path.join(OUT, "jpeg_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(json.dumps(meta))


if __name__ == "__main__":
    main()
