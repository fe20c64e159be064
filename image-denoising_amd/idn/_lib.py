"""ctypes binding of the HIP C-ABI library (include/idn.h -> idn/libidn_hip.so).

The library is the only compute path: there is no CPU fallback.  If the .so is missing (not
built) or cannot be loaded, every op raises immediately.

`variant("tuning")` swaps in the tools-only build idn/libidn_hip_tuning.so for the duration of a
`with` block (tests that compare a kernel's alternative forms, selected by its tuning knobs); the
product never loads it.
"""
from __future__ import annotations

import contextlib
import ctypes
import threading
from pathlib import Path

LIB_PATH = Path(__file__).resolve().parent / "libidn_hip.so"
ABI_VERSION = 6  # IDN_ABI_VERSION of include/idn.h that SIGNATURES binds
VARIANTS = {"tuning": Path(__file__).resolve().parent / "libidn_hip_tuning.so"}

_c_u8p = ctypes.c_void_p
_c_f64p = ctypes.c_void_p
_c_int = ctypes.c_int
_c_i64 = ctypes.c_int64
_c_u64 = ctypes.c_uint64
_c_dbl = ctypes.c_double
_c_size = ctypes.c_size_t
_c_vp = ctypes.c_void_p

# name -> (restype, argtypes); must match include/idn.h exactly
SIGNATURES = {
    "idn_abi_version": (_c_int, []),
    "idn_version": (ctypes.c_char_p, []),
    "idn_last_error": (ctypes.c_char_p, []),
    "idn_gaussian_blur_u8": (_c_int, [_c_u8p, _c_u8p, _c_int, _c_int, _c_int, _c_int, _c_i64, _c_int, _c_vp]),
    "idn_box_blur_u8": (_c_int, [_c_u8p, _c_u8p, _c_int, _c_int, _c_int, _c_int, _c_i64, _c_int, _c_vp]),
    "idn_median_blur_u8": (_c_int, [_c_u8p, _c_u8p, _c_int, _c_int, _c_int, _c_int, _c_i64, _c_int, _c_vp]),
    "idn_bilateral_u8": (_c_int, [_c_u8p, _c_u8p, _c_int, _c_int, _c_int, _c_int, _c_i64, _c_int, _c_dbl, _c_dbl, _c_vp]),
    "idn_noise_u8": (_c_int, [_c_u8p, _c_u8p, _c_f64p, _c_int, _c_int, _c_int, _c_int, _c_i64, _c_int,
                              _c_dbl, _c_dbl, _c_u64, _c_u64, _c_f64p, _c_vp, _c_size, _c_vp]),
    "idn_noise_workspace_size": (_c_size, [_c_int, _c_int]),
    "idn_poisson_levels": (_c_int, [_c_vp, _c_vp, _c_vp]),
    "idn_jpeg_info": (_c_int, [_c_vp, _c_size, _c_vp, _c_vp, _c_vp]),
    "idn_jpeg_orientation": (_c_int, [_c_vp, _c_size, _c_vp]),
    "idn_jpeg_workspace_size": (_c_size, [_c_vp, _c_vp, _c_int, _c_int]),
    "idn_jpeg_decode_u8": (_c_int, [_c_vp, _c_vp, _c_int, _c_vp, _c_int, _c_int, _c_i64, _c_int,
                                    _c_vp, _c_size, _c_vp]),
    "idn_noise_ids_u8": (_c_int, [_c_u8p, _c_u8p, _c_f64p, _c_int, _c_int, _c_int, _c_int, _c_i64,
                                  _c_int, _c_dbl, _c_dbl, _c_u64, _c_vp, _c_vp, _c_size, _c_vp]),
    "idn_noise_slots_u8": (_c_int, [_c_u8p, _c_u8p, _c_f64p, _c_int, _c_int, _c_int, _c_int, _c_i64,
                                    _c_int, _c_dbl, _c_dbl, _c_u64, _c_vp, _c_vp, _c_vp, _c_size,
                                    _c_vp]),
    "idn_noise_ycc_u8": (_c_int, [_c_u8p, _c_u8p, _c_f64p, _c_int, _c_int, _c_int, _c_int, _c_dbl,
                                  _c_dbl, _c_u64, _c_u64, _c_vp, _c_f64p, _c_vp, _c_vp]),
    "idn_noise_add_u8": (_c_int, [_c_u8p, _c_u8p, _c_f64p, _c_int, _c_int, _c_int, _c_int, _c_i64, _c_int,
                                  _c_dbl, _c_dbl, _c_u64, _c_u64, _c_f64p, _c_vp, _c_size, _c_vp]),
    "idn_noise_add_workspace_size": (_c_size, [_c_int, _c_int, _c_int, _c_int, _c_int]),
    "idn_noise_add_ids_u8": (_c_int, [_c_u8p, _c_u8p, _c_f64p, _c_int, _c_int, _c_int, _c_int,
                                      _c_i64, _c_int, _c_dbl, _c_dbl, _c_u64, _c_vp, _c_vp, _c_size,
                                      _c_vp]),
    "idn_periodic_pattern_u8": (_c_int, [_c_u8p, _c_int, _c_int, _c_int, _c_dbl, _c_vp]),
    "idn_add_pattern_u8": (_c_int, [_c_u8p, _c_u8p, _c_u8p, _c_int, _c_int, _c_int, _c_int, _c_i64, _c_vp]),
    "idn_add_pattern_slots_u8": (_c_int, [_c_u8p, _c_u8p, _c_u8p, _c_int, _c_int, _c_int, _c_int, _c_vp,
                                          _c_vp]),
    "idn_copy_slots_u8": (_c_int, [_c_u8p, _c_u8p, _c_int, _c_i64, _c_vp, _c_vp]),
    "idn_quant_u8": (_c_int, [_c_u8p, _c_u8p, _c_u8p, _c_int, _c_int, _c_int, _c_i64, _c_int, _c_u64,
                              _c_u64, _c_vp, _c_vp, _c_vp, _c_vp, _c_size, _c_vp]),
    "idn_quant_workspace_size": (_c_size, [_c_int, _c_int]),
    "idn_bgr2lab_u8": (_c_int, [_c_u8p, _c_u8p, _c_int, _c_int, _c_int, _c_i64, _c_vp]),
    "idn_lab2bgr_u8": (_c_int, [_c_u8p, _c_u8p, _c_int, _c_int, _c_int, _c_i64, _c_vp]),
    "idn_gaussian_blob_f32": (_c_int, [_c_u8p, _c_vp, _c_int, _c_int, _c_int, _c_int, _c_i64, _c_int,
                                       ctypes.POINTER(ctypes.c_double), _c_vp]),
    "idn_copy_u8": (_c_int, [_c_u8p, _c_u8p, _c_i64, _c_int, _c_vp]),
    "idn_wavelet_denoise_u8": (_c_int, [_c_u8p, _c_f64p, _c_u8p, _c_vp, _c_int, _c_int, _c_int, _c_i64,
                                        _c_int, _c_int, _c_vp, _c_size, _c_vp]),
    "idn_wavelet_denoise_ycc": (_c_int, [_c_f64p, _c_vp, _c_u8p, _c_vp, _c_int, _c_int, _c_int,
                                         _c_int, _c_int, _c_vp, _c_size, _c_vp]),
    "idn_wavelet_workspace_size": (_c_size, [_c_int, _c_int, _c_int, _c_int, _c_int]),
    "idn_wavelet_stats_offset": (_c_size, [_c_int, _c_int, _c_int, _c_int, _c_int]),
    "idn_gaussian_blur_f64": (_c_int, [_c_vp, _c_vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_vp]),
    "idn_box_blur_f64": (_c_int, [_c_vp, _c_vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_vp]),
    "idn_shader_u8": (_c_int, [_c_u8p, _c_u8p, _c_int, _c_int, _c_int, _c_int, _c_i64, _c_dbl, _c_vp]),
    "idn_bloom_u8": (_c_int, [_c_u8p, _c_u8p, _c_int, _c_int, _c_int, _c_int, _c_i64, _c_vp, _c_vp, _c_int,
                              _c_vp, _c_vp]),
    "idn_blob_from_f64": (_c_int, [_c_vp, _c_vp, _c_int, _c_int, _c_int, _c_int, _c_int,
                                   ctypes.POINTER(ctypes.c_double), _c_int, _c_vp]),
    "idn_resize_linear_f32": (_c_int, [_c_vp, _c_vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_dbl,
                                       _c_dbl, _c_vp]),
    "idn_blob_f32": (_c_int, [_c_u8p, _c_vp, _c_int, _c_int, _c_int, _c_int, _c_i64, _c_int, _c_int,
                              ctypes.POINTER(ctypes.c_double), _c_int, _c_vp]),
}

_lock = threading.Lock()
_lib = None


class IdnError(RuntimeError):
    """A C-ABI call returned a negative idn_status."""


def _open(path: Path, required: bool):
    if not path.exists():
        raise IdnError(
            f"{path} is missing: build it with `python -m idn._build` "
            "(or __graft_entry__.build()); idn has no CPU fallback")
    lib = ctypes.CDLL(str(path))
    ver = getattr(lib, "idn_abi_version", None)
    got = None
    if ver is not None:
        ver.restype, ver.argtypes = ctypes.c_int, []
        got = ver()
    if got != ABI_VERSION:
        raise IdnError(f"{path.name} has C-ABI version {got}, this binding needs {ABI_VERSION}: "
                       "rebuild it with `python -m idn._build`")
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            if required:
                raise IdnError(f"{path.name} does not export {name}")
            continue
        fn.restype = res
        fn.argtypes = args
    return lib


def load(required: bool = False):
    """Load libidn_hip.so and bind the declared symbols (raises if the library is missing;
    with required=True also if any symbol of include/idn.h is not exported)."""
    global _lib
    with _lock:
        if _lib is None:
            _lib = _open(LIB_PATH, required)
    return _lib


_variants: dict = {}


@contextlib.contextmanager
def variant(name: str):
    """Route every op through a variant build of the library inside the block (tests only)."""
    global _lib
    with _lock:
        if name not in _variants:
            _variants[name] = _open(VARIANTS[name], True)
        prev, _lib = _lib, _variants[name]
    try:
        yield _lib
    finally:
        with _lock:
            _lib = prev


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().idn_last_error()
        raise IdnError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
