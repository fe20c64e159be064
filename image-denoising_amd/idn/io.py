"""Image loading for the drop-in path: cv2.imread semantics (BGR uint8 HxWx3).

The reference reads every image with cv2.imread (lib/model/test.py:191,
lib/roi_data_layer/minibatch.py:85), i.e. OpenCV 3.4.2 over IJG libjpeg 9d (requirements.txt:74,
89).  `imread` uses OpenCV when it is importable.  Without it, a JPEG is decoded by the GPU decoder
(`imread_gpu`: bit-exact with libjpeg 9d) and returned as a host array -- never by PIL, whose
libjpeg-turbo differs from 9d by up to tens of LSB on subsampled files; a JPEG the GPU decoder
does not take raises IdnError.  Other (lossless) formats go through PIL, flipped to BGR.

`imread_gpu` is the GPU decode front-end: JPEG files are decoded on the
device (idn_jpeg_decode_u8), bit-exact with the reference's pinned IJG libjpeg 9d by default or
with libjpeg-turbo (mode="turbo"), images of one size in one launch; files the decoder does not
take raise IdnError (no CPU fallback inside the product).  Like OpenCV 3.4.2's imread, each JPEG
is turned by its EXIF orientation (APP1 IFD0 tag 0x0112: flips / transposes; idn_jpeg_orientation)
unless orientation=False (IMREAD_IGNORE_ORIENTATION).  PNG and the other lossless formats never
carry it in the form OpenCV 3.4.2's EXIF reader walks (it reads JPEG markers), so `_imread_pil`
leaves them as stored.
"""
from __future__ import annotations

import numpy as np


def imread(path) -> np.ndarray:
    """cv2.imread(path) (IMREAD_COLOR) as a host uint8 BGR HxWx3 array."""
    try:
        import cv2
    except ImportError:
        cv2 = None
    if cv2 is not None:
        im = cv2.imread(str(path))
        if im is None:
            raise FileNotFoundError(path)
        return im
    with open(path, "rb") as f:
        head = f.read(3)
    if head[:2] == b"\xff\xd8":  # JPEG: the libjpeg 9d decode, on the GPU
        return imread_gpu([path])[0].cpu().numpy()
    return _imread_pil(path)


def _imread_pil(path) -> np.ndarray:
    """a lossless format through PIL, as OpenCV's decoders return it with IMREAD_COLOR: 8-bit BGR,
    alpha dropped, palettes expanded.  Samples deeper than 8 bits keep their high byte, as
    grfmt_png.cpp's png_set_strip_16 does (PIL's own 16-bit grayscale -> RGB conversion would clip
    them at 255 instead); PIL already unpacks 16-bit RGB(A) to its high bytes."""
    from PIL import Image
    with Image.open(path) as im:
        if im.mode in ("I;16", "I;16B", "I;16L", "I"):
            g = np.asarray(im).astype(np.int64)
            if im.mode == "I" and g.max(initial=0) > 0xFFFF:
                raise ValueError(f"{path}: 32-bit samples are not an OpenCV IMREAD_COLOR input")
            g = (g >> 8).astype(np.uint8)
            return np.ascontiguousarray(np.repeat(g[..., None], 3, -1))
        rgb = np.asarray(im.convert("RGB"))
    return np.ascontiguousarray(rgb[..., ::-1])


def imread_gpu(paths, mode: str = "libjpeg9", orientation: bool = True):
    """cv2.imread for a list of JPEG paths, decoded on the GPU: a list of (h, w, 3) uint8 BGR
    device tensors in input order, each turned by its EXIF orientation (orientation=False:
    IMREAD_IGNORE_ORIENTATION); files of the same output size share one decode launch."""
    from . import ops
    datas = []
    for p in paths:
        with open(p, "rb") as f:
            datas.append(f.read())
    groups = {}
    for i, d in enumerate(datas):
        groups.setdefault(ops.jpeg_info(d, orientation)[:2], []).append(i)
    out = [None] * len(datas)
    for idx in groups.values():
        dec = ops.jpeg_decode([datas[i] for i in idx], mode=mode, orientation=orientation)
        for k, i in enumerate(idx):
            out[i] = dec[k]
    return out
