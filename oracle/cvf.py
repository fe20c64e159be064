"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by the product path).

numpy restatement of the OpenCV 3.4.2 floating-point paths the reference reaches:

  gaussian_blur_f64  cv2.GaussianBlur on the float64 output of random_noise (the plain-noise
                     branches, e.g. lib/roi_data_layer/minibatch.py:159 gaus_blur after the
                     float64 'gaussian' branch; lib/model/test.py fallback path).  sepFilter2D:
                     RowFilter<double> (taps left to right) then SymmColumnFilter<double>
                     (ky0*c + ky1*(r+1 + r-1) + ...), BORDER_REFLECT_101.
  blur_f64           cv2.blur on float64: boxFilter's RowSum (running sum s += S[i+k] - S[i]) and
                     ColumnSum (SUM += rows; s0 = SUM + new; D = s0 * 1/9; SUM = s0 - old).
  resize_linear_f32  cv2.resize(im, None, None, fx, fy, INTER_LINEAR) on the float32 blob image
                     (lib/utils/blob.py:44, lib/model/test.py:74): resizeGeneric's float
                     coefficients fx = (float)((dx+0.5)*scale - 0.5), clamped at the borders,
                     HResizeLinear (copy past xmax) and VResizeLinear, mul-then-add in float32.

cv2 is not importable here: the restatement follows the OpenCV 3.4.2 sources' algorithm; parity of
these three against a real cv2 build is UNPINNED.
"""
from __future__ import annotations

import numpy as np

_G = {3: np.array([0.25, 0.5, 0.25]), 5: np.array([0.0625, 0.25, 0.375, 0.25, 0.0625])}


def _reflect101_idx(n: int, r: int) -> np.ndarray:
    idx = np.arange(-r, n + r)
    if n == 1:
        return np.zeros_like(idx)
    while True:
        lo = idx < 0
        hi = idx >= n
        if not (lo.any() or hi.any()):
            return idx
        idx = np.where(lo, -idx, idx)
        idx = np.where(idx >= n, 2 * (n - 1) - idx, idx)


def _nhwc64(img):
    a = np.asarray(img, np.float64)
    sq = a.ndim == 3
    return (a[None] if sq else a), sq


def gaussian_blur_f64(img, ksize: int) -> np.ndarray:
    a, sq = _nhwc64(img)
    n, h, w, c = a.shape
    k = _G[ksize]
    r = ksize // 2
    ex = a[:, :, _reflect101_idx(w, r), :]
    rows = k[0] * ex[:, :, 0:w, :]
    for j in range(1, ksize):
        rows = rows + k[j] * ex[:, :, j:j + w, :]
    ey = rows[:, _reflect101_idx(h, r), :, :]
    out = k[r] * ey[:, r:r + h]
    for t in range(1, r + 1):
        out = out + k[r + t] * (ey[:, r + t:r + t + h] + ey[:, r - t:r - t + h])
    return out[0] if sq else out


def blur_f64(img, ksize: int = 3) -> np.ndarray:
    a, sq = _nhwc64(img)
    n, h, w, c = a.shape
    r = ksize // 2
    ex = a[:, :, _reflect101_idx(w, r), :]
    rs = np.empty((n, h, w, c))
    s = np.zeros((n, h, c))
    for i in range(ksize):
        s = s + ex[:, :, i, :]
    rs[:, :, 0] = s
    for x in range(1, w):
        s = s + (ex[:, :, x - 1 + ksize, :] - ex[:, :, x - 1, :])
        rs[:, :, x] = s
    ey = rs[:, _reflect101_idx(h, r)]
    out = np.empty_like(rs)
    SUM = np.zeros((n, w, c))
    for i in range(ksize - 1):
        SUM = SUM + ey[:, i]
    scale = 1.0 / (ksize * ksize)
    for y in range(h):
        s0 = SUM + ey[:, y + ksize - 1]
        out[:, y] = s0 * scale
        SUM = s0 - ey[:, y]
    return out[0] if sq else out


def _lin_tab(dsize: int, ssize: int, scale: float):
    d = np.arange(dsize, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    lo = s < 0
    f[lo] = 0
    s[lo] = 0
    hi = s >= ssize - 1
    f[hi] = 0
    s[hi] = ssize - 1
    s1 = np.minimum(s + 1, ssize - 1)
    return s, s1, (np.float32(1) - f).astype(np.float32), f, hi


def resize_linear_f32(img, fx: float, fy: float) -> np.ndarray:
    a = np.asarray(img, np.float32)
    h, w = a.shape[:2]
    oh, ow = int(round(h * fy)), int(round(w * fx))
    if (oh, ow) == (h, w):
        return a.copy()
    x0, x1, ax0, ax1, xcopy = _lin_tab(ow, w, 1.0 / fx)
    y0, y1, by0, by1, _ = _lin_tab(oh, h, 1.0 / fy)
    hz = a[:, x0] * ax0[None, :, None] + a[:, x1] * ax1[None, :, None]
    hz[:, xcopy] = a[:, x0[xcopy]]
    out = hz[y0] * by0[:, None, None] + hz[y1] * by1[:, None, None]
    return out.astype(np.float32)
