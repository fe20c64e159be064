"""Image loading for the drop-in path: cv2.imread semantics (BGR uint8 HxWx3).

The reference reads every image with cv2.imread (lib/model/test.py:191,
lib/roi_data_layer/minibatch.py:85).  OpenCV is used when importable; otherwise the file is
decoded with PIL and flipped to BGR (libjpeg builds can differ by a few LSB between the two
decoders; parity tests therefore feed both sides the same decoded pixels).

`imread_gpu` is the GPU decode front-end: baseline JPEG files are decoded on
the device (idn_jpeg_decode_u8), bit-exact with the reference's pinned IJG libjpeg 9d
(requirements.txt:74) by default or with libjpeg-turbo (mode="turbo"), images of one size in one
launch; files the decoder does not take raise IdnError (no CPU fallback inside the product).
"""
from __future__ import annotations

import numpy as np


def imread(path) -> np.ndarray:
    try:
        import cv2
    except ImportError:
        cv2 = None
    if cv2 is not None:
        im = cv2.imread(str(path))
        if im is None:
            raise FileNotFoundError(path)
        return im
    from PIL import Image
    with Image.open(path) as im:
        rgb = np.asarray(im.convert("RGB"))
    return np.ascontiguousarray(rgb[..., ::-1])


def imread_gpu(paths, mode: str = "libjpeg9"):
    """cv2.imread for a list of JPEG paths, decoded on the GPU: a list of (h, w, 3) uint8 BGR
    device tensors in input order; same-size files share one decode launch."""
    from . import ops
    datas = []
    for p in paths:
        with open(p, "rb") as f:
            datas.append(f.read())
    groups = {}
    for i, d in enumerate(datas):
        groups.setdefault(ops.jpeg_info(d)[:2], []).append(i)
    out = [None] * len(datas)
    for idx in groups.values():
        dec = ops.jpeg_decode([datas[i] for i in idx], mode=mode)
        for k, i in enumerate(idx):
            out[i] = dec[k]
    return out
