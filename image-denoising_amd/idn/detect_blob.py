"""Drop-in for the test-side path of lib/model/test.py: the noise / denoise body of test_net's
per-image loop (189-1831) and the blob builders _get_image_blob (49-83) / _get_blobs (85-90).

    im = apply_noise(img, noise)          # replaces test.py:193-1831 for one image
    blobs, im_scales = _get_blobs(im)     # test.py:85, then net.test_image(...)

or, with the decode front-end on the GPU too (cv2.imread at test.py:191):

    im = apply_noise(path, noise, decode="gpu")

mode='test_v0' (default) reproduces test.py as-is (sap/quant add no noise, gaussian picks a random
level and returns float64, only the 'wavelet' post hook is live, unknown strings fall to
gaussian_var0.1 + 3x3 mean on the float image).
"""
from __future__ import annotations

import random as _random
from types import SimpleNamespace

import numpy as np

from pathlib import Path

from . import blobs as _blob
from . import io as _io
from .pipeline import Preprocessor

cfg = SimpleNamespace(
    PIXEL_MEANS=np.array([[[102.9801, 115.9465, 122.7717]]]),
    RNG_SEED=3,
    TEST=SimpleNamespace(SCALES=(600,), MAX_SIZE=1000),
)
_PRE = {}


def apply_noise(img, noise: str, mode: str = "test_v0", image_id: int = 0,
                noise_rng: str = "philox", as_tensor: bool = False, decode: str = "host"):
    """One image through the reference's noise + denoise recipe on the GPU (uint8 or float64).

    img: the cv2.imread image (numpy / device tensor) or a file path, read by cv2.imread
    semantics: decode="host" (PIL / cv2 on the host) or decode="gpu" (the GPU JPEG decoder,
    bit-exact with the pinned libjpeg 9d; no CPU fallback: an unsupported file raises)."""
    if decode not in ("host", "gpu"):
        raise ValueError("decode must be 'host' or 'gpu'")
    if isinstance(img, (str, Path)):
        img = _io.imread_gpu([img])[0] if decode == "gpu" else _io.imread(img)
    key = (noise, mode, noise_rng)
    if key not in _PRE:
        _PRE[key] = Preprocessor(noise, mode, seed=cfg.RNG_SEED, rng=_random, noise_rng=noise_rng)
    outs, _ = _PRE[key](_blob._to_device(img)[None], image_ids=[image_id])
    return outs[0] if as_tensor else _blob._to_host(outs[0])


def _get_image_blob(im, as_tensor: bool = False):
    """Converts an image into a network input (test.py:49)."""
    processed_ims, im_scale_factors = [], []
    for target_size in cfg.TEST.SCALES:
        f, im_scale = _blob.prep_im_for_blob(im, cfg.PIXEL_MEANS, target_size, cfg.TEST.MAX_SIZE,
                                             as_tensor=True)
        im_scale_factors.append(im_scale)
        processed_ims.append(f)
    blob = _blob.im_list_to_blob(processed_ims, as_tensor=as_tensor)
    return blob, np.array(im_scale_factors)


def _get_blobs(im, as_tensor: bool = False):
    """Convert an image and RoIs within that image into network inputs (test.py:85)."""
    blobs = {}
    blobs["data"], im_scale_factors = _get_image_blob(im, as_tensor=as_tensor)
    return blobs, im_scale_factors
