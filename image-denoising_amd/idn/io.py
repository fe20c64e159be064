"""Image loading for the drop-in path: cv2.imread semantics (BGR uint8 HxWx3).

The reference reads every image with cv2.imread (lib/model/test.py:191,
lib/roi_data_layer/minibatch.py:85).  OpenCV is used when importable; otherwise the file is
decoded with PIL and flipped to BGR (libjpeg builds can differ by a few LSB between the two
decoders; parity tests therefore feed both sides the same decoded pixels).  A GPU JPEG decode
front-end is a SURVEY §8(f) "next" row.
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
