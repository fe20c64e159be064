"""idn — MI355X-native image noise-injection + denoising filter bank.

Drop-in for the preprocessing hot path of mahesh-kashyap-ml/image-denoising (the noise closures
and denoise hooks of lib/roi_data_layer/minibatch.py and lib/model/test.py, and
lib/utils/blob.py), computed by hand-written HIP kernels for gfx950 behind a C-ABI
(include/idn.h).  See DESIGN.md.
"""
from ._lib import IdnError, LIB_PATH  # noqa: F401
from . import ops  # noqa: F401
from .ops import (  # noqa: F401
    gaussian_blur, blur, median_blur, bilateral_filter, random_noise, periodic_pattern,
    add_pattern, periodic_noise, blob,
)

__version__ = "0.1.0"
