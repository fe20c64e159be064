"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by the product path).

ctypes front-end for oracle/filters.c, the plain-C restatement of the OpenCV 3.4.2 8-bit filters
the reference calls (cv2.GaussianBlur / blur / medianBlur / bilateralFilter; call sites listed in
filters.c).  Arrays are numpy uint8 (H,W,C) or (N,H,W,C), C-contiguous.
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

_DIR = Path(__file__).resolve().parent
_SO = _DIR / "_build" / "liboracle.so"
_lib = None


def build() -> Path:
    newest = max((_DIR / f).stat().st_mtime for f in ("filters.c", "baseline_fast.c", "Makefile"))
    if not _SO.exists() or _SO.stat().st_mtime < newest:
        subprocess.run(["make", "-s", "-C", str(_DIR)], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(str(_SO))
        u8p = ctypes.c_void_p
        i = ctypes.c_int
        i64 = ctypes.c_int64
        d = ctypes.c_double
        for name in ("oracle_gaussian_u8", "oracle_box_u8", "oracle_median_u8",
                     "baseline_gaussian_u8"):
            f = getattr(L, name)
            f.argtypes = [u8p, u8p, i, i, i, i, i64, i]
            f.restype = None
        L.oracle_bilateral_u8.argtypes = [u8p, u8p, i, i, i, i, i64, i, d, d]
        L.oracle_bilateral_u8.restype = None
        L.oracle_bilateral_f32.argtypes = [u8p, u8p, i, i, i, i, i64, i, d, d]
        L.oracle_bilateral_f32.restype = None
        L.oracle_matmul3_fma.argtypes = [u8p, u8p, i64, u8p, u8p, u8p]
        L.oracle_matmul3_fma.restype = None
        _lib = L
    return _lib


def _nhwc(img: np.ndarray):
    a = np.ascontiguousarray(img)
    if a.dtype != np.uint8:
        raise TypeError(f"oracle filters take uint8 images, got {a.dtype}")
    squeeze = False
    if a.ndim == 2:
        a = a[None, :, :, None]
        squeeze = 2
    elif a.ndim == 3:
        a = a[None]
        squeeze = 3
    n, h, w, c = a.shape
    return a, (n, h, w, c), squeeze


def _unsq(out, squeeze):
    if squeeze == 2:
        return out[0, :, :, 0]
    if squeeze == 3:
        return out[0]
    return out


def _run(name, img, *extra):
    a, (n, h, w, c), sq = _nhwc(img)
    out = np.empty_like(a)
    getattr(lib(), name)(a.ctypes.data, out.ctypes.data, n, h, w, c, w * c, *extra)
    return _unsq(out, sq)


def gaussian_blur(img: np.ndarray, ksize: int) -> np.ndarray:
    """cv2.GaussianBlur(img, (ksize, ksize), 0) for ksize in {3, 5}."""
    assert ksize in (3, 5)
    return _run("oracle_gaussian_u8", img, ksize)


def gaussian_blur_fast(img: np.ndarray, ksize: int) -> np.ndarray:
    """The timed CPU baseline (baseline_fast.c): the same cv2.GaussianBlur result computed the
    way OpenCV's 8-bit path does it (separable, 16-bit SIMD row sums, OpenMP)."""
    assert ksize in (3, 5)
    return _run("baseline_gaussian_u8", img, ksize)


def blur(img: np.ndarray, ksize: int = 3) -> np.ndarray:
    """cv2.blur(img, (ksize, ksize))."""
    return _run("oracle_box_u8", img, ksize)


def median_blur(img: np.ndarray, ksize: int) -> np.ndarray:
    """cv2.medianBlur(img, ksize)."""
    return _run("oracle_median_u8", img, ksize)


def bilateral_filter(img: np.ndarray, d: int, sigma_color: float, sigma_space: float) -> np.ndarray:
    """cv2.bilateralFilter(img, d, sigma_color, sigma_space, borderType=cv2.BORDER_CONSTANT)."""
    return _run("oracle_bilateral_u8", img, d, float(sigma_color), float(sigma_space))


def bilateral_prefilter_f32(img, d, sigma_color, sigma_space) -> np.ndarray:
    """fp64-accumulated bilateral value before cvRound (float32), shape (N,H,W,C)."""
    a, (n, h, w, c), sq = _nhwc(img)
    out = np.empty((n, h, w, c), np.float32)
    lib().oracle_bilateral_f32(a.ctypes.data, out.ctypes.data, n, h, w, c, w * c, d,
                               float(sigma_color), float(sigma_space))
    return _unsq(out, sq)


def matmul3_fma(x: np.ndarray, M: np.ndarray, pre=(0.0, 0.0, 0.0), post=(0.0, 0.0, 0.0)) -> np.ndarray:
    """(x - pre) @ M.T + post with numpy/OpenBLAS's fma-chain rounding (see filters.c)."""
    a = np.ascontiguousarray(x, np.float64)
    out = np.empty_like(a)
    Mc = np.ascontiguousarray(M, np.float64)
    pr = np.ascontiguousarray(pre, np.float64)
    po = np.ascontiguousarray(post, np.float64)
    lib().oracle_matmul3_fma(a.ctypes.data, out.ctypes.data, a.size // 3, Mc.ctypes.data,
                             pr.ctypes.data, po.ctypes.data)
    return out
