"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by the product path).

numpy restatement of the two OpenCV 3.4.2 colour conversions the reference's `quant` noise makes
(lib/model/test.py:594,606 / lib/roi_data_layer/minibatch.py:496,508):

  cv2.cvtColor(img_u8, cv2.COLOR_BGR2LAB)   RGB2Lab_b   (imgproc/src/color_lab.cpp)
  cv2.cvtColor(lab_u8, cv2.COLOR_LAB2BGR)   Lab2RGB_b -> Lab2RGBinteger (enableBitExactness)

OpenCV 3.4.x computes both 8-bit conversions in integer arithmetic from tables that
initLabTabs() builds once with its softfloat / softdouble types (IEEE binary32 / binary64 with
correct rounding for + - * /).  The tables are rebuilt here with numpy float32 / float64
arithmetic in the same operation order; cbrt / pow come from the C library and are rounded to
binary32, which can differ from OpenCV's own softfloat cbrt / softdouble pow by an ulp and so
move a table entry whose scaled value sits within about 1e-3 of a rounding tie.  cv2 is not
installable in this container, so parity of this restatement vs cv2 is UNPINNED.

  bgr2lab(img)    uint8 (..., 3) BGR -> uint8 (..., 3) L, a, b (8-bit scaling: L*255/100, +128)
  lab2bgr(lab)    uint8 (..., 3) L, a, b -> uint8 (..., 3) BGR
  tables()        the integer tables and coefficients (shared with the tests and the kernels'
                  constant check)
"""
from __future__ import annotations

from functools import lru_cache

import numpy as np

f32 = np.float32
LAB_SHIFT = 12            # xyz_shift
GAMMA_SHIFT = 3
LAB_SHIFT2 = LAB_SHIFT + GAMMA_SHIFT
CBRT_TAB_SIZE_B = 256 * 3 // 2 * (1 << GAMMA_SHIFT)   # 3072
INV_GAMMA_TAB_SIZE = 4096
BASE = 1 << 14            # lab_base_shift
MIN_AB = -8145            # minABvalue
AB_TAB_SIZE = BASE * 9 // 4

# sRGB2XYZ_D65 / XYZ2sRGB_D65 / D65 (color.hpp), as the double values of the decimal constants
SRGB2XYZ = (0.412453, 0.357580, 0.180423, 0.212671, 0.715160, 0.072169, 0.019334, 0.119193,
            0.950227)
XYZ2SRGB = (3.240479, -1.53715, -0.498535, -0.969256, 1.875991, 0.041556, 0.055648, -0.204043,
            1.057311)
D65 = (0.950456, 1.0, 1.088754)


def _round_even(x) -> np.ndarray:
    """cvRound on softfloat / softdouble: round to nearest, ties to even."""
    return np.rint(np.asarray(x, np.float64)).astype(np.int64)


def _gamma(x32: np.ndarray) -> np.ndarray:
    """applyGamma(softfloat x) in softdouble, returned as softfloat."""
    xd = x32.astype(np.float64)
    thr = 809.0 / 20000.0
    low = 323.0 / 25.0
    shift = 11.0 / 200.0
    power = 12.0 / 5.0
    out = np.where(xd <= thr, xd / low, np.power((xd + shift) / (1.0 + shift), power))
    return out.astype(f32)


def _inv_gamma(x32: np.ndarray) -> np.ndarray:
    """applyInvGamma(softfloat x) in softdouble, returned as softfloat."""
    xd = x32.astype(np.float64)
    thr = 7827.0 / 2500000.0
    low = 323.0 / 25.0
    shift = 11.0 / 200.0
    power = 12.0 / 5.0
    out = np.where(xd <= thr, xd * low, np.power(xd, 1.0 / power) * (1.0 + shift) - shift)
    return out.astype(f32)


@lru_cache(maxsize=1)
def tables():
    f255 = f32(255)
    lthresh = f32(216) / f32(24389)
    lscale = f32(841) / f32(108)
    lbias = f32(16) / f32(116)
    i256 = np.arange(256)
    # sRGBGammaTab_b[i] = cvRound(255*8 * applyGamma(i / 255))
    x = i256.astype(f32) / f255
    gamma_b = _round_even(f32(255 * (1 << GAMMA_SHIFT)) * _gamma(x)).astype(np.int64)
    # sRGBInvGammaTab_b[i] = cvRound(255 * applyInvGamma(i / 4096))
    xi = f32(1.0) / f32(INV_GAMMA_TAB_SIZE) * np.arange(INV_GAMMA_TAB_SIZE).astype(f32)
    inv_gamma_b = _round_even(f255 * _inv_gamma(xi.astype(f32))).astype(np.int64)
    # LabCbrtTab_b[i] = cvRound(2^15 * (x < lthresh ? x*lscale + lbias : cbrt(x))), x = i/(255*8)
    cb_scale = f32(1.0) / (f255 * f32(1 << GAMMA_SHIFT))
    xc = (cb_scale * np.arange(CBRT_TAB_SIZE_B).astype(f32)).astype(f32)
    lin = (xc.astype(np.float64) * np.float64(lscale) + np.float64(lbias)).astype(f32)  # mulAdd
    cbr = np.cbrt(xc.astype(np.float64)).astype(f32)
    fx = np.where(xc < lthresh, lin, cbr).astype(f32)
    cbrt_b = _round_even(f32(1 << LAB_SHIFT2) * fx).astype(np.int64)
    # LabToYF_b: (y, ify) per 8-bit L
    y = np.zeros(256, np.int64)
    ify = np.zeros(256, np.int64)
    for i in range(256):
        if i <= 20:
            y[i] = _round_even(f32(i * BASE * 20 * 9) / f32(17 * 29 * 29 * 29))
            ify[i] = _round_even(f32(BASE) * (f32(16) / f32(116) + f32(i * 5) / f32(3 * 17 * 29)))
        else:
            fy = f32(f32(i * 100 * BASE) / f32(255 * 116) + f32(16 * BASE) / f32(116))
            ify[i] = _round_even(fy)
            y[i] = _round_even(f32(f32(fy * fy) * fy) / f32(BASE * BASE))
    # abToXZ_b (plain C int arithmetic: division truncates toward zero)
    ab = np.zeros(AB_TAB_SIZE, np.int64)
    for k, i in enumerate(range(MIN_AB, AB_TAB_SIZE + MIN_AB)):
        if i <= 3390:
            q = abs(i * 108) // 841
            ab[k] = (q if i * 108 >= 0 else -q) - BASE * 16 // 116 * 108 // 841
        else:
            ab[k] = i * i // BASE * i // BASE
    # RGB2Lab_b coefficients for BGR input (blueIdx = 0): row i = X, Y, Z; columns B, G, R
    lshift = float(1 << LAB_SHIFT)
    c_fwd = np.zeros(9, np.int64)
    for i in range(3):
        c = SRGB2XYZ[i * 3: i * 3 + 3]
        c_fwd[i * 3 + 2] = _round_even(lshift * c[0] / D65[i])   # R
        c_fwd[i * 3 + 1] = _round_even(lshift * c[1] / D65[i])   # G
        c_fwd[i * 3 + 0] = _round_even(lshift * c[2] / D65[i])   # B
    # Lab2RGBinteger coefficients: output rows R, G, B; columns X, Y, Z
    c_inv = np.zeros(9, np.int64)
    for i in range(3):
        for j in range(3):
            c_inv[j * 3 + i] = _round_even(lshift * XYZ2SRGB[i + j * 3] * D65[i])
    return dict(gamma_b=gamma_b, inv_gamma_b=inv_gamma_b, cbrt_b=cbrt_b, y_b=y, ify_b=ify,
                ab_to_xz=ab, c_fwd=c_fwd, c_inv=c_inv)


def _descale(x, n):
    return (x + (1 << (n - 1))) >> n


def bgr2lab(img: np.ndarray) -> np.ndarray:
    """cv2.cvtColor(img, COLOR_BGR2LAB) for uint8 BGR (RGB2Lab_b::operator())."""
    t = tables()
    a = np.asarray(img)
    assert a.dtype == np.uint8 and a.shape[-1] == 3
    g = t["gamma_b"]
    B, G, R = (g[a[..., k].astype(np.int64)] for k in range(3))
    C = t["c_fwd"]
    cb = t["cbrt_b"]
    fX = cb[_descale(B * C[0] + G * C[1] + R * C[2], LAB_SHIFT)]
    fY = cb[_descale(B * C[3] + G * C[4] + R * C[5], LAB_SHIFT)]
    fZ = cb[_descale(B * C[6] + G * C[7] + R * C[8], LAB_SHIFT)]
    Lscale = (116 * 255 + 50) // 100
    Lshift = -((16 * 255 * (1 << LAB_SHIFT2) + 50) // 100)
    L = _descale(Lscale * fY + Lshift, LAB_SHIFT2)
    aa = _descale(500 * (fX - fY) + 128 * (1 << LAB_SHIFT2), LAB_SHIFT2)
    bb = _descale(200 * (fY - fZ) + 128 * (1 << LAB_SHIFT2), LAB_SHIFT2)
    return np.stack([np.clip(v, 0, 255) for v in (L, aa, bb)], axis=-1).astype(np.uint8)


def lab2bgr(lab: np.ndarray) -> np.ndarray:
    """cv2.cvtColor(lab, COLOR_LAB2BGR) for uint8 Lab (Lab2RGBinteger::process)."""
    t = tables()
    a = np.asarray(lab)
    assert a.dtype == np.uint8 and a.shape[-1] == 3
    L, A, Bv = (a[..., k].astype(np.int64) for k in range(3))
    y = t["y_b"][L]
    ify = t["ify_b"][L]
    adiv = A * BASE // 500 - 128 * BASE // 500
    bdiv = Bv * BASE // 200 - 128 * BASE // 200
    x = t["ab_to_xz"][ify + adiv - MIN_AB]
    z = t["ab_to_xz"][ify - bdiv - MIN_AB]
    C = t["c_inv"]
    shift = LAB_SHIFT + (14 - 12)  # lab_shift + (base_shift - inv_gamma_shift)
    out = []
    for row in (2, 1, 0):  # B, G, R rows of the XYZ->sRGB matrix
        v = _descale(C[row * 3] * x + C[row * 3 + 1] * y + C[row * 3 + 2] * z, shift)
        v = np.clip(v, 0, INV_GAMMA_TAB_SIZE - 1)
        out.append(t["inv_gamma_b"][v])
    return np.clip(np.stack(out, axis=-1), 0, 255).astype(np.uint8)


def quantize_apply(img: np.ndarray, centers: np.ndarray):
    """The reference's quant given fitted centres: labels = argmin of
    ||c||^2 - 2 x.c (sklearn _labels_inertia, float64), quant = centres.astype(uint8)[labels],
    LAB->BGR.  Returns (bgr_u8, labels, lab)."""
    lab = bgr2lab(img)
    X = lab.reshape(-1, 3).astype(np.float64)
    c = np.asarray(centers, np.float64)
    d = (c * c).sum(1)[None, :] - 2.0 * (X @ c.T)
    labels = np.argmin(d, axis=1)
    quant = c.astype(np.uint8)[labels].reshape(lab.shape)
    return lab2bgr(quant), labels.reshape(lab.shape[:-1]), lab


def inertia(lab: np.ndarray, centers: np.ndarray) -> float:
    """sum over pixels of the squared distance to the nearest centre (sklearn's inertia_)."""
    X = lab.reshape(-1, 3).astype(np.float64)
    c = np.asarray(centers, np.float64)
    d = ((X[:, None, :] - c[None, :, :]) ** 2).sum(-1)
    return float(d.min(1).sum())
