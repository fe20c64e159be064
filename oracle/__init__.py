"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference's hot-path arithmetic (OpenCV filters in C, skimage / numpy
float64 arithmetic in numpy, the wavelet denoiser in numpy).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package, and only as the
checker or the timed CPU baseline.  The product (image-denoising_amd/idn) never imports it and
fails loudly when its HIP library is missing.
"""
from . import automold, cv, cvf, cvlab, sk, wavelet  # noqa: F401
