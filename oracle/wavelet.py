"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by the product path).

numpy restatement of the wavelet denoiser the reference calls:

  denoise_wavelet(im, method='BayesShrink', mode='soft', wavelet='bior1.5',
                  multichannel=True, convert2ycbcr=True)          lib/model/test.py:197-201,1807-1810
                                                                  minibatch.py:1653-1656
  denoise_wavelet(im, ..., wavelet_levels=3)  (default 'db1')     minibatch_before_curvelet.py:85-87

with scikit-image 0.14.2's wrapper semantics (the two colour matmuls use numpy/OpenBLAS's fma-chain
rounding, reproduced in C by oracle/filters.c:oracle_matmul3_fma, so zero sets of the finest dd do
not depend on the host BLAS kernel) (requirements.txt:160): img_as_float, rgb2ycbcr on
the (BGR-as-RGB) data, per channel min/max normalisation, `_wavelet_threshold` (pywt wavedecn,
'symmetric' mode, level default max(dwt_max_level - 3, 1), sigma = median(|finest dd| != 0) /
0.6744897501960817, BayesShrink thresholds var / sqrt(max(mean(d^2) - var, eps)) per detail band,
soft thresholding, waverecn, crop), inner clip to [0, 1], de-normalise, ycbcr2rgb, outer clip to
[0, 1].  The discrete wavelet transform restates PyWavelets 1.x's C kernels
(downsampling_convolution / upsampling_convolution_valid_sf, symmetric extension).

Pinned by tests/golden/golden.npz: pywt.wavedecn / waverecn coefficient arrays and the full
denoiser on crops and on a 600x1000 image (tests/test_oracle.py).
"""
from __future__ import annotations

import numpy as np

_S = 0.7071067811865476
_B1 = 0.016572815184059706
_B2 = 0.12153397801643785
FILTERS = {
    # name: (dec_lo, dec_hi, rec_lo, rec_hi)  (PyWavelets filter banks)
    "db1": ([_S, _S], [-_S, _S], [_S, _S], [_S, -_S]),
    "bior1.5": ([_B1, -_B1, -_B2, _B2, _S, _S, _B2, -_B2, -_B1, _B1],
                [-0.0, 0.0, -0.0, 0.0, -_S, _S, -0.0, 0.0, -0.0, 0.0],
                [0.0, 0.0, 0.0, 0.0, _S, _S, 0.0, 0.0, 0.0, 0.0],
                [_B1, _B1, -_B2, -_B2, _S, -_S, _B2, _B2, -_B1, -_B1]),
}
FILTERS["haar"] = FILTERS["db1"]
NORM_PPF75 = 0.6744897501960817  # scipy.stats.norm.ppf(0.75)
YCBCR_FROM_RGB = np.array([[65.481, 128.553, 24.966],
                           [-37.797, -74.203, 112.0],
                           [112.0, -93.786, -18.214]])
RGB_FROM_YCBCR = np.linalg.inv(YCBCR_FROM_RGB)
YCBCR_OFFSET = np.array([16.0, 128.0, 128.0])


def dwt_max_level(n: int, flen: int) -> int:
    if flen <= 1 or n < flen - 1:
        return 0
    return int(n // (flen - 1)).bit_length() - 1


def _sym_index(i, n):
    """half-sample symmetric extension index (pywt 'symmetric'), any overshoot"""
    period = 2 * n
    i = np.mod(i, period)
    return np.where(i < n, i, period - 1 - i)


def dwt1(x: np.ndarray, w: str, axis: int):
    lo, hi = (np.asarray(f, np.float64) for f in FILTERS[w][:2])
    F = len(lo)
    x = np.moveaxis(x, axis, -1)
    N = x.shape[-1]
    nout = (N + F - 1) // 2
    # output o uses full-convolution index i = 2o + 1: y[i] = sum_j f[j] x[i - j]
    i = 2 * np.arange(nout) + 1
    idx = _sym_index(i[:, None] - np.arange(F)[None, :], N)  # (nout, F)
    g = x[..., idx]  # (..., nout, F)
    a = g @ lo
    d = g @ hi
    return np.moveaxis(a, -1, axis), np.moveaxis(d, -1, axis)


def idwt1(a: np.ndarray, d: np.ndarray, w: str, axis: int):
    rlo, rhi = (np.asarray(f, np.float64) for f in FILTERS[w][2:])
    F = len(rlo)
    a = np.moveaxis(a, axis, -1)
    d = np.moveaxis(d, axis, -1)
    N = a.shape[-1]
    h = F // 2
    i = np.arange(h - 1, N)  # stage 2 only: every filter tap overlaps an input sample
    idx = i[:, None] - np.arange(h)[None, :]  # (m, h)
    ga, gd = a[..., idx], d[..., idx]
    even = ga @ rlo[0::2] + gd @ rhi[0::2]
    odd = ga @ rlo[1::2] + gd @ rhi[1::2]
    out = np.stack([even, odd], axis=-1).reshape(*even.shape[:-1], 2 * even.shape[-1])
    return np.moveaxis(out, -1, axis)


def dwtn(x: np.ndarray, w: str):
    coeffs = [("", x)]
    for axis in range(x.ndim):
        nxt = []
        for key, arr in coeffs:
            a, d = dwt1(arr, w, axis)
            nxt += [(key + "a", a), (key + "d", d)]
        coeffs = nxt
    return dict(coeffs)


def idwtn(coeffs: dict, w: str):
    ndim = len(next(iter(coeffs)))
    for axis in reversed(range(ndim)):
        nxt = {}
        keys = sorted({k[:axis] for k in coeffs})
        for key in keys:
            nxt[key] = idwt1(coeffs[key + "a"], coeffs[key + "d"], w, axis)
        coeffs = nxt
    return coeffs[""]


def wavedecn(x: np.ndarray, w: str, level: int):
    out = []
    a = x
    for _ in range(level):
        c = dwtn(a, w)
        a = c.pop("a" * x.ndim)
        out.append(c)
    return [a] + out[::-1]


def waverecn(coeffs, w: str):
    a = coeffs[0]
    for i, d in enumerate(coeffs[1:]):
        if i > 0:  # _match_coeff_dims: crop the approximation to the detail shape
            ref = next(iter(d.values()))
            a = a[tuple(slice(s) for s in ref.shape)]
        c = dict(d)
        c["a" * a.ndim] = a
        a = idwtn(c, w)
    return a


def wavelet_threshold(img2d: np.ndarray, w: str, levels=None) -> np.ndarray:
    """skimage _wavelet_threshold(method='BayesShrink', mode='soft', sigma=None)."""
    if levels is None:
        F = len(FILTERS[w][0])
        levels = max(min(dwt_max_level(s, F) for s in img2d.shape) - 3, 1)
    co = wavedecn(img2d, w, levels)
    finest = co[-1]["d" * img2d.ndim]
    nz = finest[np.nonzero(finest)]
    sigma = np.median(np.abs(nz)) / NORM_PPF75
    var = sigma ** 2
    eps = np.finfo(np.float64).eps
    den = [co[0]]
    for lev in co[1:]:
        dl = {}
        for k, d in lev.items():
            dvar = np.mean(d * d)
            t = var / np.sqrt(max(dvar - var, eps))
            mag = np.abs(d)
            with np.errstate(divide="ignore", invalid="ignore"):
                s = 1 - t / mag
            s = np.clip(s, 0, None)
            s = np.where(mag == 0, 0.0, s)
            dl[k] = d * s
        den.append(dl)
    rec = waverecn(den, w)
    return rec[tuple(slice(s) for s in img2d.shape)]


def denoise_wavelet(img, wavelet: str = "bior1.5", levels=None) -> np.ndarray:
    """skimage 0.14.2 denoise_wavelet(img, method='BayesShrink', mode='soft', wavelet=wavelet,
    multichannel=True, convert2ycbcr=True, wavelet_levels=levels) -> float64 [0, 1]."""
    from .cv import matmul3_fma
    x = img.astype(np.float64) * (1.0 / 255.0) if img.dtype == np.uint8 else np.asarray(img, np.float64)
    out = matmul3_fma(x, YCBCR_FROM_RGB, post=YCBCR_OFFSET)  # rgb2ycbcr
    for i in range(3):
        mn, mx = out[..., i].min(), out[..., i].max()
        ch = (out[..., i] - mn) / (mx - mn)
        ch = np.clip(wavelet_threshold(ch, wavelet, levels), 0, 1)
        out[..., i] = ch * (mx - mn) + mn
    out = matmul3_fma(out, RGB_FROM_YCBCR, pre=YCBCR_OFFSET)  # ycbcr2rgb
    return np.clip(out, 0, 1)
