"""Tensor-level ops over the HIP C-ABI (device tensors in, device tensors out).

Every function takes uint8 images shaped (H, W, C) or (N, H, W, C) living on a ROCm device
(torch "cuda" tensors) and launches on torch's current stream.  Names and argument meaning follow
the OpenCV / scikit-image calls the reference makes on its preprocessing path:

  gaussian_blur(x, ksize)                 cv2.GaussianBlur(x, (ksize, ksize), 0)
  blur(x, ksize=3)                        cv2.blur(x, (ksize, ksize))
  median_blur(x, ksize)                   cv2.medianBlur(x, ksize)
  bilateral_filter(x, d, sc, ss)          cv2.bilateralFilter(x, d, sc, ss, BORDER_CONSTANT)
  random_noise(x, mode, ...)              skimage.util.random_noise (+ U8 cast)
  periodic_pattern / add_pattern          add_periodic_noise's linspace/sin pattern, cv2.add
  denoise_wavelet(x, wavelet, levels)     skimage.restoration.denoise_wavelet (0.14.2 wrapper)
  blob(x, ...)                            lib/utils/blob.py prep_im_for_blob + im_list_to_blob

There is no CPU path: a CPU tensor raises, a missing library raises.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np
import torch

from . import _lib

PIXEL_MEANS = (102.9801, 115.9465, 122.7717)  # lib/model/config.py:252 (BGR)

NOISE_KINDS = {"gaussian": 0, "speckle": 1, "s&p": 2, "sap": 2, "poisson": 3}
WAVELETS = {"db1": 0, "haar": 0, "bior1.5": 1}


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _as_batch(x: torch.Tensor, name: str) -> Tuple[torch.Tensor, bool]:
    if not isinstance(x, torch.Tensor):
        raise TypeError(f"{name}: expected a torch.Tensor, got {type(x).__name__}")
    if x.device.type != "cuda":
        raise ValueError(f"{name}: idn runs on the GPU only; got a {x.device} tensor "
                         "(move it with .cuda(); there is no CPU fallback)")
    squeeze = False
    if x.dim() == 3:
        x = x.unsqueeze(0)
        squeeze = True
    if x.dim() != 4:
        raise ValueError(f"{name}: expected (H,W,C) or (N,H,W,C), got shape {tuple(x.shape)}")
    return x, squeeze


def _u8_batch(x: torch.Tensor, name: str) -> Tuple[torch.Tensor, bool]:
    x, sq = _as_batch(x, name)
    if x.dtype != torch.uint8:
        raise TypeError(f"{name}: expected uint8 images, got {x.dtype}")
    if not x.is_contiguous():
        x = x.contiguous()
    return x, sq


def _finish(out: torch.Tensor, squeeze: bool) -> torch.Tensor:
    return out[0] if squeeze else out


def _filter(fn_name: str, x: torch.Tensor, *args, out: Optional[torch.Tensor] = None):
    xb, sq = _u8_batch(x, fn_name)
    n, h, w, c = xb.shape
    y = torch.empty_like(xb) if out is None else out.view(n, h, w, c)
    lib = _lib.load()
    rc = getattr(lib, fn_name)(xb.data_ptr(), y.data_ptr(), n, h, w, c, w * c, *args, _stream())
    _lib.check(rc, fn_name)
    return _finish(y, sq)


def gaussian_blur(x: torch.Tensor, ksize: int = 5, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """cv2.GaussianBlur(x, (ksize, ksize), 0); ksize in {3, 5}; bit-exact."""
    return _filter("idn_gaussian_blur_u8", x, int(ksize), out=out)


def blur(x: torch.Tensor, ksize: int = 3, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """cv2.blur(x, (ksize, ksize)); ksize 3; bit-exact."""
    return _filter("idn_box_blur_u8", x, int(ksize), out=out)


def median_blur(x: torch.Tensor, ksize: int = 3, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """cv2.medianBlur(x, ksize); ksize in {3, 5}; bit-exact."""
    return _filter("idn_median_blur_u8", x, int(ksize), out=out)


def bilateral_filter(x: torch.Tensor, d: int = 9, sigma_color: float = 20.0,
                     sigma_space: float = 100.0, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """cv2.bilateralFilter(x, d, sigma_color, sigma_space, borderType=BORDER_CONSTANT)."""
    return _filter("idn_bilateral_u8", x, int(d), float(sigma_color), float(sigma_space), out=out)


# ---- noise generators ------------------------------------------------------------------------

def _empty_like_img(xb: torch.Tensor, dtype) -> torch.Tensor:
    return torch.empty(xb.shape, dtype=dtype, device=xb.device)


def _ids_tensor(image_ids, n: int, device) -> torch.Tensor:
    """device uint64 (int64 storage) array of n image ids for the *_ids_u8 entry points.  An
    int64 tensor already on the device is used as is (no host copy, no sync; the caller owns its
    validity); anything else is checked on the host and copied over."""
    if isinstance(image_ids, torch.Tensor) and image_ids.device == device \
            and image_ids.dtype == torch.int64:
        t = image_ids.reshape(-1)
        if t.numel() != n:
            raise ValueError(f"image_ids has {t.numel()} entries for a batch of {n}")
        return t.contiguous()
    t = torch.as_tensor(image_ids, dtype=torch.int64).reshape(-1)
    if t.numel() != n:
        raise ValueError(f"image_ids has {t.numel()} entries for a batch of {n}")
    if bool((t < 0).any()):
        raise ValueError("image_ids must be non-negative")
    return t.to(device).contiguous()


def random_noise(x: torch.Tensor, mode: str = "gaussian", *, mean: float = 0.0, var: float = 0.01,
                 amount: float = 0.05, salt_vs_pepper: float = 0.5, seed: int = 0,
                 offset: int = 0, replay: Optional[torch.Tensor] = None, out: str = "u8",
                 out_u8: Optional[torch.Tensor] = None, image_ids=None, slots=None):
    """skimage.util.random_noise(x, mode, ...) on a uint8 batch, plus the caller's U8 cast.

    out="u8"   -> (255 * random_noise(...)).astype(np.uint8)   (denoise-branch input)
    out="f64"  -> random_noise(...) as float64 in [0, 1]        ("plain" branch result)
    out="both" -> (u8, f64)
    replay: None draws from the Philox stream keyed by (seed, offset + image index); otherwise the
    random field numpy would have drawn (gaussian/speckle: N(mean, sqrt(var)) field of x.shape;
    s&p: float64 [2, *x.shape] random_sample fields for `flipped` then `salted`; poisson: the
    Poisson draws), which makes the result bit-exact with the reference.
    image_ids: optional per-image ids (Philox stream only) instead of offset + index -- one launch
    for any subset of a batch, drawing what per-image calls with offset = id would.
    slots: with image_ids, an int64 device tensor of batch positions: only images x[slots] are
    noised, written to out_u8[slots] (out="u8", out_u8 required, the rest of out_u8 untouched) --
    a mixed batch's per-type group with no gather / scatter of its images.
    """
    if slots is not None:
        return _random_noise_slots(x, mode, mean, var, amount, salt_vs_pepper, seed, out, out_u8,
                                   image_ids, slots)
    kind = NOISE_KINDS.get(mode.lower())
    if kind is None:
        raise ValueError(f"random_noise: unsupported mode {mode!r}; supported: {sorted(NOISE_KINDS)}")
    xb, sq = _u8_batch(x, "random_noise")
    n, h, w, c = xb.shape
    want_u8 = out in ("u8", "both")
    want_f64 = out in ("f64", "both")
    if not (want_u8 or want_f64):
        raise ValueError("random_noise: out must be 'u8', 'f64' or 'both'")
    y8 = (out_u8.view(n, h, w, c) if out_u8 is not None else _empty_like_img(xb, torch.uint8)) if want_u8 else None
    y64 = _empty_like_img(xb, torch.float64) if want_f64 else None
    if kind in (0, 1):
        p0, p1 = float(mean), float(var)
    elif kind == 2:
        p0, p1 = float(amount), float(salt_vs_pepper)
    else:
        p0 = p1 = 0.0
    rp = None
    if replay is not None:
        rp = replay
        if rp.device != xb.device or rp.dtype != torch.float64:
            raise ValueError("random_noise: replay must be a float64 tensor on the same device")
        need = (2 if kind == 2 else 1) * xb.numel()
        if rp.numel() != need:
            raise ValueError(f"random_noise: replay has {rp.numel()} elements, expected {need}")
        rp = rp.contiguous()
    lib = _lib.load()
    ws = None
    ws_bytes = lib.idn_noise_workspace_size(kind, n)
    if ws_bytes:
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=xb.device)
    if image_ids is not None:
        if rp is not None:
            raise ValueError("random_noise: image_ids applies to the Philox stream, not to replay")
        ids = _ids_tensor(image_ids, n, xb.device)
        rc = lib.idn_noise_ids_u8(xb.data_ptr(), y8.data_ptr() if y8 is not None else None,
                                  y64.data_ptr() if y64 is not None else None, n, h, w, c, w * c,
                                  kind, p0, p1, int(seed) & (2 ** 64 - 1), ids.data_ptr(),
                                  ws.data_ptr() if ws is not None else None, ws_bytes, _stream())
        _lib.check(rc, "idn_noise_ids_u8")
    else:
        rc = lib.idn_noise_u8(xb.data_ptr(), y8.data_ptr() if y8 is not None else None,
                              y64.data_ptr() if y64 is not None else None, n, h, w, c, w * c,
                              kind, p0, p1, int(seed) & (2 ** 64 - 1), int(offset),
                              rp.data_ptr() if rp is not None else None,
                              ws.data_ptr() if ws is not None else None, ws_bytes, _stream())
        _lib.check(rc, "idn_noise_u8")
    if out == "u8":
        return _finish(y8, sq)
    if out == "f64":
        return _finish(y64, sq)
    return _finish(y8, sq), _finish(y64, sq)


def ycc_fusable(x: torch.Tensor) -> bool:
    """random_noise_ycc takes this batch: uint8, 3 channels, an even pixel count per image"""
    return x.dtype == torch.uint8 and x.shape[-1] == 3 and (x.shape[-3] * x.shape[-2]) % 2 == 0


def random_noise_ycc(x: torch.Tensor, mode: str = "gaussian", *, mean: float = 0.0,
                     var: float = 0.01, seed: int = 0, offset: int = 0,
                     replay: Optional[torch.Tensor] = None, image_ids=None):
    """random_noise(x, mode, out='f64') for gaussian / speckle, fused with the wavelet's colour
    range (idn_noise_ycc_u8; lib/model/test.py:1678-1684 -> 1807-1810: the float64 image goes
    straight into denoise_wavelet).  Returns (the float64 image -- the same values as
    random_noise(..., out='f64') -- and an (N, 6) int64 device tensor of per-image YCbCr min / max
    keys for denoise_wavelet(..., ycc_keys=...))."""
    kind = NOISE_KINDS.get(mode.lower())
    if kind not in (0, 1):
        raise ValueError(f"random_noise_ycc: gaussian or speckle only (got {mode!r})")
    xb, sq = _u8_batch(x, "random_noise_ycc")
    n, h, w, c = xb.shape
    if c != 3:
        raise ValueError("random_noise_ycc: needs 3 channels")
    xb = xb.contiguous()
    y64 = _empty_like_img(xb, torch.float64)
    keys = torch.empty((n, 6), dtype=torch.int64, device=xb.device)
    rp = None
    if replay is not None:
        if replay.device != xb.device or replay.dtype != torch.float64 or replay.numel() != xb.numel():
            raise ValueError("random_noise_ycc: replay must be a float64 field of x's shape on its device")
        rp = replay.contiguous()
    ids = None
    if image_ids is not None:
        if rp is not None:
            raise ValueError("random_noise_ycc: image_ids applies to the Philox stream, not to replay")
        ids = _ids_tensor(image_ids, n, xb.device)
    rc = _lib.load().idn_noise_ycc_u8(xb.data_ptr(), None, y64.data_ptr(), n, h, w, kind,
                                      float(mean), float(var), int(seed) & (2 ** 64 - 1),
                                      int(offset), ids.data_ptr() if ids is not None else None,
                                      rp.data_ptr() if rp is not None else None, keys.data_ptr(),
                                      _stream())
    _lib.check(rc, "idn_noise_ycc_u8")
    return _finish(y64, sq), keys


def _slots_tensor(slots, device) -> torch.Tensor:
    """The caller owns slot validity (0 <= slot < batch size, as for device image-id tensors):
    checking a device tensor's values would cost a host sync per launch."""
    if not (isinstance(slots, torch.Tensor) and slots.device == device
            and slots.dtype == torch.int64):
        raise ValueError("slots must be an int64 tensor on the batch's device")
    return slots.reshape(-1).contiguous()


def _random_noise_slots(x, mode, mean, var, amount, salt_vs_pepper, seed, out, out_u8, image_ids,
                        slots):
    kind = NOISE_KINDS.get(mode.lower())
    if kind is None:
        raise ValueError(f"random_noise: unsupported mode {mode!r}; supported: {sorted(NOISE_KINDS)}")
    if out != "u8" or out_u8 is None or image_ids is None:
        raise ValueError("random_noise: slots needs out='u8', out_u8 and image_ids")
    xb, _ = _u8_batch(x, "random_noise")
    nb, h, w, c = xb.shape
    if not (isinstance(out_u8, torch.Tensor) and out_u8.dtype == torch.uint8
            and out_u8.device == xb.device and out_u8.is_contiguous()
            and tuple(out_u8.shape) in ((nb, h, w, c), (h, w, c) if nb == 1 else ())):
        raise ValueError("random_noise: slots needs out_u8 = a contiguous uint8 tensor shaped "
                         "like x on x's device")
    y8 = out_u8.view(nb, h, w, c)
    sl = _slots_tensor(slots, xb.device)
    n = sl.numel()
    ids = _ids_tensor(image_ids, n, xb.device)
    if kind in (0, 1):
        p0, p1 = float(mean), float(var)
    elif kind == 2:
        p0, p1 = float(amount), float(salt_vs_pepper)
    else:
        p0 = p1 = 0.0
    lib = _lib.load()
    ws_bytes = lib.idn_noise_workspace_size(kind, n)
    ws = _workspace(ws_bytes, xb.device) if ws_bytes else None
    rc = lib.idn_noise_slots_u8(xb.data_ptr(), y8.data_ptr(), None, n, h, w, c, w * c, kind, p0, p1,
                                int(seed) & (2 ** 64 - 1), ids.data_ptr(), sl.data_ptr(),
                                ws.data_ptr() if ws is not None else None, ws_bytes, _stream())
    _lib.check(rc, "idn_noise_slots_u8")
    return out_u8


ADD_NOISE_KINDS = {"uniform": 4, "gamma": 5, "rayleigh": 6, "brownian": 7}
GAMMA_SHAPE = 1.99  # a = 1.99 in every gamma closure (lib/model/test.py:1303)


def noise_add(x: torch.Tensor, mode: str, level: float, *, seed: int = 0, offset: int = 0,
              replay: Optional[torch.Tensor] = None, out: str = "u8",
              out_u8: Optional[torch.Tensor] = None, shape: float = GAMMA_SHAPE, image_ids=None):
    """The reference's own additive noises (lib/model/test.py:767-1572), u8 batch in:
      uniform  level = high:  out = img_as_float(x) + np.random.uniform(0, high)
      gamma    level = scale: out = x + scipy.stats.gamma.rvs(1.99, scale=level)
      rayleigh level = scale: out = x + scipy.stats.rayleigh.rvs(scale=level)
      brownian level = dt:    u8 = cv2.add(img, U8(255 * cumsum-walk)), f64 = the walk B
    cv2.add(float64, float64) does not clip: out="f64" is the unclipped sum (what train_v0's plain
    branches return), out="u8" is (255 * out).astype(np.uint8) with its modulo-256 wrap.
    replay: numpy's unit draws (random_sample / standard_gamma(1.99) / sqrt(chisquare(2)) /
    for brownian the normals with element e holding z[e-1]), float64 of x's shape.
    image_ids: optional per-image ids (Philox stream only), as in random_noise."""
    kind = ADD_NOISE_KINDS.get(mode.lower())
    if kind is None:
        raise ValueError(f"noise_add: unsupported mode {mode!r}; supported: {sorted(ADD_NOISE_KINDS)}")
    xb, sq = _u8_batch(x, "noise_add")
    n, h, w, c = xb.shape
    want_u8 = out in ("u8", "both")
    want_f64 = out in ("f64", "both")
    if not (want_u8 or want_f64):
        raise ValueError("noise_add: out must be 'u8', 'f64' or 'both'")
    y8 = (out_u8.view(n, h, w, c) if out_u8 is not None else _empty_like_img(xb, torch.uint8)) if want_u8 else None
    y64 = _empty_like_img(xb, torch.float64) if want_f64 else None
    p0, p1 = (float(shape), float(level)) if kind == 5 else (float(level), 0.0)
    rp = None
    if replay is not None:
        if replay.device != xb.device or replay.dtype != torch.float64 or replay.numel() != xb.numel():
            raise ValueError("noise_add: replay must be float64, on the same device, one value per element")
        rp = replay.contiguous()
    lib = _lib.load()
    ws_bytes = lib.idn_noise_add_workspace_size(kind, n, h, w, c)
    ws = _workspace(ws_bytes, xb.device) if ws_bytes else None
    if image_ids is not None:
        if rp is not None:
            raise ValueError("noise_add: image_ids applies to the Philox stream, not to replay")
        ids = _ids_tensor(image_ids, n, xb.device)
        rc = lib.idn_noise_add_ids_u8(xb.data_ptr(), y8.data_ptr() if y8 is not None else None,
                                      y64.data_ptr() if y64 is not None else None, n, h, w, c,
                                      w * c, kind, p0, p1, int(seed) & (2 ** 64 - 1),
                                      ids.data_ptr(), ws.data_ptr() if ws is not None else None,
                                      ws_bytes, _stream())
        _lib.check(rc, "idn_noise_add_ids_u8")
    else:
        rc = lib.idn_noise_add_u8(xb.data_ptr(), y8.data_ptr() if y8 is not None else None,
                                  y64.data_ptr() if y64 is not None else None, n, h, w, c, w * c,
                                  kind, p0, p1, int(seed) & (2 ** 64 - 1), int(offset),
                                  rp.data_ptr() if rp is not None else None,
                                  ws.data_ptr() if ws is not None else None, ws_bytes, _stream())
        _lib.check(rc, "idn_noise_add_u8")
    if out == "u8":
        return _finish(y8, sq)
    if out == "f64":
        return _finish(y64, sq)
    return _finish(y8, sq), _finish(y64, sq)


_PATTERN_CACHE: dict = {}


def periodic_pattern(h: int, w: int, c: int, amplitude: float, device=None) -> torch.Tensor:
    """U8(255*sin(linspace(-A, A, h*w*c))).reshape(h, w, c); cached per (h, w, c, A, device)."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    key = (h, w, c, float(amplitude), str(dev))
    pat = _PATTERN_CACHE.get(key)
    if pat is None:
        pat = torch.empty((h, w, c), dtype=torch.uint8, device=dev)
        rc = _lib.load().idn_periodic_pattern_u8(pat.data_ptr(), h, w, c, float(amplitude), _stream())
        _lib.check(rc, "idn_periodic_pattern_u8")
        _PATTERN_CACHE[key] = pat
    return pat


def add_pattern(x: torch.Tensor, pattern: torch.Tensor, out: Optional[torch.Tensor] = None,
                slots=None) -> torch.Tensor:
    """cv2.add(x, pattern) (u8 saturating), pattern broadcast over the batch.  slots (int64 device
    tensor, out required): only images x[slots] -> out[slots]."""
    xb, sq = _u8_batch(x, "add_pattern")
    n, h, w, c = xb.shape
    if tuple(pattern.shape) != (h, w, c) or pattern.dtype != torch.uint8:
        raise ValueError(f"add_pattern: pattern must be uint8 {(h, w, c)}, got {tuple(pattern.shape)}")
    if slots is not None:
        if out is None:
            raise ValueError("add_pattern: slots needs out")
        sl = _slots_tensor(slots, xb.device)
        rc = _lib.load().idn_add_pattern_slots_u8(xb.data_ptr(), pattern.contiguous().data_ptr(),
                                                  out.data_ptr(), sl.numel(), h, w, c,
                                                  sl.data_ptr(), _stream())
        _lib.check(rc, "idn_add_pattern_slots_u8")
        return out
    y = torch.empty_like(xb) if out is None else out.view(n, h, w, c)
    rc = _lib.load().idn_add_pattern_u8(xb.data_ptr(), pattern.contiguous().data_ptr(), y.data_ptr(),
                                        n, h, w, c, w * c, _stream())
    _lib.check(rc, "idn_add_pattern_u8")
    return _finish(y, sq)


def periodic_noise(x: torch.Tensor, amplitude: float, out: Optional[torch.Tensor] = None,
                   slots=None) -> torch.Tensor:
    """add_periodic_noise: cv2.add(img, U8(255*sin(linspace(-A, A, img.size))).reshape(h,w,3))."""
    xb, _ = _as_batch(x, "periodic_noise")
    _, h, w, c = xb.shape
    return add_pattern(x, periodic_pattern(h, w, c, amplitude, xb.device), out=out, slots=slots)


def copy_slots(x: torch.Tensor, out: torch.Tensor, slots) -> torch.Tensor:
    """out[slots] = x[slots] for a uint8 batch (the noise-free members of a mixed batch)."""
    xb, _ = _u8_batch(x, "copy_slots")
    if out.shape != x.shape or out.dtype != torch.uint8 or not out.is_contiguous():
        raise ValueError("copy_slots: out must be a contiguous uint8 tensor shaped like x")
    sl = _slots_tensor(slots, xb.device)
    per_img = xb[0].numel() if xb.shape[0] else 1
    rc = _lib.load().idn_copy_slots_u8(xb.data_ptr(), out.data_ptr(), sl.numel(), per_img,
                                       sl.data_ptr(), _stream())
    _lib.check(rc, "idn_copy_slots_u8")
    return out


# ---- fused steps -------------------------------------------------------------------------------

FILTERS = {"gaus_blur": 0, "mean": 1}


def noise_filter(x: torch.Tensor, mode: str, filter: str, ksize: int, *, var: float = 0.01,
                 amount: float = 0.05, salt_vs_pepper: float = 0.5, seed: int = 0,
                 offset: int = 0, image_ids=None, out: Optional[torch.Tensor] = None,
                 form: str = "serial"):
    """random_noise(x, mode, ...) -> U8 -> cv2.GaussianBlur (filter 'gaus_blur') or cv2.blur
    ('mean'); the result is identical in every form (Philox u8 stream keyed by (seed, image id)).
      form 'serial'    the noise launch, then the filter launch (the default: fastest measured,
                       profiles/r02/README.md -- the noise is VALU-bound; a one-pass fused LDS-ring
                       form measured slower and was removed in round 3)
      form 'pipelined' the batch in chunks: the noise of chunk k+1 (VALU-bound) runs on a side
                       stream beside the filter of chunk k (HBM-bound), whose input is still in
                       the 256 MB Infinity Cache"""
    if form == "pipelined":
        return _noise_filter_pipelined(x, mode, filter, ksize, var=var, amount=amount,
                                       salt_vs_pepper=salt_vs_pepper, seed=seed, offset=offset,
                                       image_ids=image_ids, out=out)
    if form != "serial":
        raise ValueError("noise_filter: form must be 'serial' or 'pipelined'")
    kind = NOISE_KINDS.get(mode.lower())
    if kind is None or kind == 3:
        raise ValueError(f"noise_filter: mode {mode!r} not supported (gaussian, speckle, s&p)")
    if filter not in FILTERS:
        raise ValueError(f"noise_filter: filter must be one of {sorted(FILTERS)}")
    xb, sq = _u8_batch(x, "noise_filter")
    n, h, w, c = xb.shape
    y = torch.empty_like(xb) if out is None else out.view(n, h, w, c)
    kw = dict(amount=amount, salt_vs_pepper=salt_vs_pepper) if kind == 2 else dict(var=var)
    t = random_noise(xb, mode, seed=seed, offset=offset, image_ids=image_ids, out="u8", **kw)
    return _finish((gaussian_blur if filter == "gaus_blur" else blur)(t, ksize, out=y), sq)


_PIPE_STREAMS: dict = {}


def _noise_filter_pipelined(x, mode, filter, ksize, *, var, amount, salt_vs_pepper, seed, offset,
                            image_ids, out, chunk: int = 32):
    xb, sq = _u8_batch(x, "noise_filter")
    n = xb.shape[0]
    y = torch.empty_like(xb) if out is None else out.view(xb.shape)
    main = torch.cuda.current_stream(xb.device)
    side = _PIPE_STREAMS.get(xb.device)
    if side is None:
        side = _PIPE_STREAMS[xb.device] = torch.cuda.Stream(device=xb.device)
    tmp = _workspace(xb.numel(), xb.device)[: xb.numel()].view(xb.shape)
    kw = dict(amount=amount, salt_vs_pepper=salt_vs_pepper) if mode in ("s&p", "sap") else \
        dict(var=var)
    flt = gaussian_blur if filter == "gaus_blur" else blur
    side.wait_stream(main)  # inputs / outputs are ready on the caller's stream
    ids_all = _ids_tensor(image_ids, n, xb.device) if image_ids is not None else None
    prev = None
    for lo in range(0, n, chunk):
        hi = min(lo + chunk, n)
        with torch.cuda.stream(side):
            if ids_all is None:
                random_noise(xb[lo:hi], mode, seed=seed, offset=offset + lo, out="u8",
                             out_u8=tmp[lo:hi], **kw)
            else:
                random_noise(xb[lo:hi], mode, seed=seed, image_ids=ids_all[lo:hi], out="u8",
                             out_u8=tmp[lo:hi], **kw)
            ev = torch.cuda.Event()
            ev.record(side)
        if prev is not None:
            main.wait_event(prev[2])
            flt(tmp[prev[0]:prev[1]], ksize, out=y[prev[0]:prev[1]])
        prev = (lo, hi, ev)
    if prev is not None:
        main.wait_event(prev[2])
        flt(tmp[prev[0]:prev[1]], ksize, out=y[prev[0]:prev[1]])
    side.wait_stream(main)  # tmp (shared scratch) is not reused by the side stream early
    return _finish(y, sq)


def gaussian_blob(x: torch.Tensor, ksize: int = 5, pixel_means=PIXEL_MEANS,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """blob(gaussian_blur(x, ksize)) at scale 1.0 in one pass: float32 (N, H, W, 3)
    float32(float64(v) - mean[ch]) written by the filter (idn_gaussian_blob_f32)."""
    xb, _ = _u8_batch(x, "gaussian_blob")
    n, h, w, c = xb.shape
    y = torch.empty((n, h, w, c), dtype=torch.float32, device=xb.device) if out is None else out
    m = (ctypes.c_double * 3)(*[float(v) for v in np.asarray(pixel_means, np.float64).reshape(-1)])
    rc = _lib.load().idn_gaussian_blob_f32(xb.data_ptr(), y.data_ptr(), n, h, w, c, w * c,
                                           int(ksize), m, _stream())
    if rc == -2:
        return blob(gaussian_blur(xb, ksize), pixel_means, out=y)
    _lib.check(rc, "idn_gaussian_blob_f32")
    return y


# ---- quant: colour quantisation by k-means in 8-bit Lab ----------------------------------------

def quantize(x: torch.Tensor, k: int, *, seed: int = 0, offset: int = 0, image_ids=None,
             centers: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
             return_labels: bool = False, return_centers: bool = False):
    """The reference's `quant` noise (lib/model/test.py:592-765): per image
    LAB2BGR(MiniBatchKMeans(n_clusters=k).fit(BGR2LAB(x)).cluster_centers_.astype(uint8)[labels]).

    centers None: device k-means (greedy k-means++ + Lloyd, Philox draws keyed by (seed, image
    id = offset + i or image_ids[i])).  centers (float64 (N, k, 3) on the device, e.g. sklearn's
    cluster_centers_): replay -- labels exactly as sklearn assigns them.
    Returns out, plus labels (uint8 (N, H, W)) and / or the centres used ((N, k, 3) float64)."""
    xb, sq = _u8_batch(x, "quantize")
    n, h, w, c = xb.shape
    if c != 3:
        raise ValueError("quantize: needs 3-channel BGR images")
    k = int(k)
    y = torch.empty_like(xb) if out is None else out.view(n, h, w, c)
    lab = torch.empty((n, h, w), dtype=torch.uint8, device=xb.device) if return_labels else None
    cen_out = (torch.empty((n, k, 3), dtype=torch.float64, device=xb.device)
               if return_centers else None)
    cin = None
    if centers is not None:
        if centers.device != xb.device or centers.dtype != torch.float64 or \
                tuple(centers.shape) != (n, k, 3):
            raise ValueError(f"quantize: centers must be float64 {(n, k, 3)} on the batch's device")
        cin = centers.contiguous()
    ids = _ids_tensor(image_ids, n, xb.device) if image_ids is not None else None
    lib = _lib.load()
    ws_bytes = lib.idn_quant_workspace_size(n, k)
    ws = _workspace(ws_bytes, xb.device) if ws_bytes else None
    rc = lib.idn_quant_u8(xb.data_ptr(), y.data_ptr(), lab.data_ptr() if lab is not None else None,
                          n, h, w, w * 3, k, int(seed) & (2 ** 64 - 1), int(offset),
                          ids.data_ptr() if ids is not None else None,
                          cin.data_ptr() if cin is not None else None,
                          cen_out.data_ptr() if cen_out is not None else None,
                          ws.data_ptr() if ws is not None else None, ws_bytes, _stream())
    _lib.check(rc, "idn_quant_u8")
    res = [_finish(y, sq)]
    if return_labels:
        res.append(_finish(lab, sq))
    if return_centers:
        res.append(_finish(cen_out, sq))
    return res[0] if len(res) == 1 else tuple(res)


def cvt_color_lab(x: torch.Tensor, to_lab: bool = True) -> torch.Tensor:
    """cv2.cvtColor(x, COLOR_BGR2LAB) (to_lab) or (x, COLOR_LAB2BGR) on 8-bit 3-channel images."""
    xb, sq = _u8_batch(x, "cvt_color_lab")
    n, h, w, c = xb.shape
    if c != 3:
        raise ValueError("cvt_color_lab: needs 3 channels")
    y = torch.empty_like(xb)
    fn = "idn_bgr2lab_u8" if to_lab else "idn_lab2bgr_u8"
    _lib.check(getattr(_lib.load(), fn)(xb.data_ptr(), y.data_ptr(), n, h, w, w * 3, _stream()), fn)
    return _finish(y, sq)


def copy_flat(x: torch.Tensor, out: torch.Tensor, policy: int = 0) -> torch.Tensor:
    """out <- x as one flat byte copy (the bench's copy ceiling; policy 1 = nontemporal)."""
    if x.device.type != "cuda" or out.device != x.device:
        raise ValueError("copy_flat: both tensors must be on the same GPU")
    if not (x.is_contiguous() and out.is_contiguous()) or x.nbytes != out.nbytes:
        raise ValueError("copy_flat: contiguous tensors of equal byte size required")
    rc = _lib.load().idn_copy_u8(x.data_ptr(), out.data_ptr(), x.nbytes, int(policy), _stream())
    _lib.check(rc, "idn_copy_u8")
    return out


# ---- blob epilogue -----------------------------------------------------------------------------

def blob(x: torch.Tensor, pixel_means=PIXEL_MEANS, out_hw: Optional[Tuple[int, int]] = None,
         flip: bool = False, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """prep_im_for_blob (scale 1.0) + im_list_to_blob: float32 NHWC, mean-subtracted, zero-padded."""
    xb, _ = _u8_batch(x, "blob")
    n, h, w, c = xb.shape
    oh, ow = out_hw if out_hw is not None else (h, w)
    y = torch.empty((n, oh, ow, 3), dtype=torch.float32, device=xb.device) if out is None else out
    m = (ctypes.c_double * 3)(*[float(v) for v in np.asarray(pixel_means, np.float64).reshape(-1)])
    rc = _lib.load().idn_blob_f32(xb.data_ptr(), y.data_ptr(), n, h, w, c, w * c, oh, ow, m,
                                  1 if flip else 0, _stream())
    _lib.check(rc, "idn_blob_f32")
    return y


# ---- wavelet denoise ---------------------------------------------------------------------------

_WS_CACHE: dict = {}


def _workspace(nbytes: int, device) -> torch.Tensor:
    """grow-only scratch per (device, current stream) (the C-ABI never allocates): calls on one
    stream are ordered, so they may share it; calls on two streams get separate buffers."""
    key = (str(device), torch.cuda.current_stream(device).cuda_stream)
    ws = _WS_CACHE.get(key)
    if ws is None or ws.numel() < nbytes:
        ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)
        _WS_CACHE[key] = ws
    return ws


def denoise_wavelet(x: torch.Tensor, wavelet: str = "bior1.5", levels: Optional[int] = None,
                    out: str = "u8", out_u8: Optional[torch.Tensor] = None,
                    ycc_keys: Optional[torch.Tensor] = None):
    """(255 * skimage.restoration.denoise_wavelet(x, method='BayesShrink', mode='soft',
    wavelet=wavelet, multichannel=True, convert2ycbcr=True, wavelet_levels=levels)).astype(uint8)
    with skimage 0.14.2's clipping.  x: uint8 (N,)H,W,3 or float64 (N,)H,W,3 in [0, 1].
    out: 'u8' | 'f32' (float result before the cast) | 'both'.
    ycc_keys: float64 x only -- the colour range random_noise_ycc reduced while writing x (the
    same result, one read of x fewer)."""
    wv = WAVELETS.get(wavelet)
    if wv is None:
        raise ValueError(f"denoise_wavelet: unsupported wavelet {wavelet!r} (db1/haar/bior1.5)")
    xb, sq = _as_batch(x, "denoise_wavelet")
    if xb.shape[-1] != 3:
        raise ValueError("denoise_wavelet: multichannel YCbCr path needs 3 channels")
    n, h, w, _ = xb.shape
    if xb.dtype == torch.uint8:
        src, src64 = xb.contiguous(), None
    elif xb.dtype == torch.float64:
        src, src64 = None, xb.contiguous()
    else:
        raise TypeError(f"denoise_wavelet: expected uint8 or float64, got {xb.dtype}")
    want_u8 = out in ("u8", "both")
    want_f32 = out in ("f32", "both")
    y8 = (out_u8.view(n, h, w, 3) if out_u8 is not None else
          torch.empty((n, h, w, 3), dtype=torch.uint8, device=xb.device)) if want_u8 else None
    y32 = torch.empty((n, h, w, 3), dtype=torch.float32, device=xb.device) if want_f32 else None
    lib = _lib.load()
    lv = -1 if levels is None else int(levels)
    nbytes = lib.idn_wavelet_workspace_size(n, h, w, wv, lv)
    ws = _workspace(nbytes, xb.device)
    if ycc_keys is not None:
        if src64 is None:
            raise ValueError("denoise_wavelet: ycc_keys applies to float64 input")
        if (ycc_keys.dtype != torch.int64 or ycc_keys.device != xb.device
                or tuple(ycc_keys.shape) != (n, 6)):
            raise ValueError("denoise_wavelet: ycc_keys must be the (N, 6) int64 device tensor of "
                             "random_noise_ycc")
        rc = lib.idn_wavelet_denoise_ycc(src64.data_ptr(), ycc_keys.contiguous().data_ptr(),
                                         y8.data_ptr() if y8 is not None else None,
                                         y32.data_ptr() if y32 is not None else None,
                                         n, h, w, wv, lv, ws.data_ptr(), nbytes, _stream())
        _lib.check(rc, "idn_wavelet_denoise_ycc")
        if out == "u8":
            return _finish(y8, sq)
        if out == "f32":
            return _finish(y32, sq)
        return _finish(y8, sq), _finish(y32, sq)
    rc = lib.idn_wavelet_denoise_u8(src.data_ptr() if src is not None else None,
                                    src64.data_ptr() if src64 is not None else None,
                                    y8.data_ptr() if y8 is not None else None,
                                    y32.data_ptr() if y32 is not None else None,
                                    n, h, w, w * 3, wv, lv, ws.data_ptr(), nbytes, _stream())
    _lib.check(rc, "idn_wavelet_denoise_u8")
    if out == "u8":
        return _finish(y8, sq)
    if out == "f32":
        return _finish(y32, sq)
    return _finish(y8, sq), _finish(y32, sq)


# ---- float64 filters, shader, bloom ------------------------------------------------------------

def _f64_batch(x: torch.Tensor, name: str):
    xb, sq = _as_batch(x, name)
    if xb.dtype != torch.float64:
        raise TypeError(f"{name}: expected float64, got {xb.dtype}")
    return xb.contiguous(), sq


def gaussian_blur_f64(x: torch.Tensor, ksize: int = 3) -> torch.Tensor:
    """cv2.GaussianBlur on a float64 image (the train_v0 post hook after a float64 noise branch)."""
    xb, sq = _f64_batch(x, "gaussian_blur_f64")
    n, h, w, c = xb.shape
    y = torch.empty_like(xb)
    _lib.check(_lib.load().idn_gaussian_blur_f64(xb.data_ptr(), y.data_ptr(), n, h, w, c, int(ksize),
                                                 _stream()), "idn_gaussian_blur_f64")
    return _finish(y, sq)


def blur_f64(x: torch.Tensor, ksize: int = 3) -> torch.Tensor:
    """cv2.blur on a float64 image (test_v0 default branch, train_v0 'mean' post hook)."""
    xb, sq = _f64_batch(x, "blur_f64")
    n, h, w, c = xb.shape
    y = torch.empty_like(xb)
    _lib.check(_lib.load().idn_box_blur_f64(xb.data_ptr(), y.data_ptr(), n, h, w, c, int(ksize),
                                            _stream()), "idn_box_blur_f64")
    return _finish(y, sq)


def shader(x: torch.Tensor, factor: float = 3.0) -> torch.Tensor:
    """add_shader: PIL ImageEnhance.Brightness(factor) of the image, returned in RGB order."""
    xb, sq = _u8_batch(x, "shader")
    n, h, w, c = xb.shape
    y = torch.empty_like(xb)
    _lib.check(_lib.load().idn_shader_u8(xb.data_ptr(), y.data_ptr(), n, h, w, c, w * c, float(factor),
                                         _stream()), "idn_shader_u8")
    return _finish(y, sq)


def bloom(x: torch.Tensor, rng=None, circles=None, **flare_kw) -> torch.Tensor:
    """add_bloom: Automold.add_sun_flare(img, flare_center=(100,100), angle=-pi/4) per image, the
    random draws taken from `rng` (default: the global `random`, like the reference), or given
    per image as `circles` = [(circles int32 [k, 8], weights float32 [k, 2]), ...] (what
    automold.sun_flare_circles returns; plans carry them, idn.noise_spec.plan(hw=...))."""
    import math
    from . import automold
    xb, sq = _u8_batch(x, "bloom")
    n, h, w, c = xb.shape
    if circles is not None:
        if len(circles) != n:
            raise ValueError(f"bloom: {len(circles)} circle sets for {n} images")
        circ = np.stack([np.asarray(a, np.int32).reshape(-1, 8) for a, _ in circles])
        wts = np.stack([np.asarray(b, np.float32).reshape(-1, 2) for _, b in circles])
    else:
        kw = dict(flare_center=(100, 100), angle=-math.pi / 4)
        kw.update(flare_kw)
        circ, wts = zip(*[automold.sun_flare_circles(h, w, rng=rng, **kw) for _ in range(n)])
        circ, wts = np.stack(circ), np.stack(wts)
    rmax = int(circ[..., 2].max()) if circ.size else 0
    spans = torch.from_numpy(automold.span_table(max(rmax, 1))).to(xb.device)
    circ_t = torch.from_numpy(np.ascontiguousarray(circ)).to(xb.device)
    wts_t = torch.from_numpy(np.ascontiguousarray(wts)).to(xb.device)
    y = torch.empty_like(xb)
    _lib.check(_lib.load().idn_bloom_u8(xb.data_ptr(), y.data_ptr(), n, h, w, c, w * c,
                                        circ_t.data_ptr(), wts_t.data_ptr(), circ.shape[1],
                                        spans.data_ptr(), _stream()), "idn_bloom_u8")
    return _finish(y, sq)


def blob_from_f64(x: torch.Tensor, pixel_means=PIXEL_MEANS, out_hw: Optional[Tuple[int, int]] = None,
                  flip: bool = False) -> torch.Tensor:
    """prep_im_for_blob on a float64 image (the reference's float64 plain-noise branches)."""
    xb, _ = _f64_batch(x, "blob_from_f64")
    n, h, w, c = xb.shape
    oh, ow = out_hw if out_hw is not None else (h, w)
    y = torch.empty((n, oh, ow, 3), dtype=torch.float32, device=xb.device)
    m = (ctypes.c_double * 3)(*[float(v) for v in np.asarray(pixel_means, np.float64).reshape(-1)])
    _lib.check(_lib.load().idn_blob_from_f64(xb.data_ptr(), y.data_ptr(), n, h, w, oh, ow, m,
                                             1 if flip else 0, _stream()), "idn_blob_from_f64")
    return y


def resize_linear(x: torch.Tensor, fx: float, fy: float) -> torch.Tensor:
    """cv2.resize(x, None, None, fx=fx, fy=fy, interpolation=cv2.INTER_LINEAR) on float32 NHWC."""
    xb, sq = _as_batch(x, "resize_linear")
    if xb.dtype != torch.float32:
        raise TypeError("resize_linear: expected float32")
    xb = xb.contiguous()
    n, h, w, c = xb.shape
    oh, ow = int(round(h * fy)), int(round(w * fx))  # cv::Size(saturate_cast<int>(...))
    if (oh, ow) == (h, w):
        return _finish(xb.clone(), sq)  # cv2.resize copies when the size is unchanged
    y = torch.empty((n, oh, ow, c), dtype=torch.float32, device=xb.device)
    _lib.check(_lib.load().idn_resize_linear_f32(xb.data_ptr(), y.data_ptr(), n, h, w, c, oh, ow,
                                                 float(fx), float(fy), _stream()),
               "idn_resize_linear_f32")
    return _finish(y, sq)


# ---- decode front-end (cv2.imread: lib/model/test.py:191, minibatch.py:85) ------------------
def _file_ptrs(files):
    bufs = [bytes(f) for f in files]
    ptrs = (ctypes.c_void_p * len(bufs))(
        *[ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p).value for b in bufs])
    lens = (ctypes.c_size_t * len(bufs))(*[len(b) for b in bufs])
    return bufs, ptrs, lens


def jpeg_orientation(data: bytes) -> int:
    """The EXIF orientation (1..8, 1 = none) cv2.imread (OpenCV 3.4.2) applies to this JPEG after
    decoding (include/idn.h idn_jpeg_orientation)."""
    lib = _lib.load()
    o = ctypes.c_int()
    buf = bytes(data)
    _lib.check(lib.idn_jpeg_orientation(ctypes.cast(ctypes.c_char_p(buf), ctypes.c_void_p),
                                        len(buf), ctypes.byref(o)), "idn_jpeg_orientation")
    return o.value


def jpeg_info(data: bytes, orientation: bool = True) -> Tuple[int, int, int]:
    """(height, width, components) of a JPEG held in memory, as cv2.imread returns it (the size
    after its EXIF orientation; orientation=False: the decoded size); IdnError if the decoder
    does not take it (lossless, hierarchical, 12-bit, ...)."""
    lib = _lib.load()
    h, w, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    buf = bytes(data)
    _lib.check(lib.idn_jpeg_info(ctypes.cast(ctypes.c_char_p(buf), ctypes.c_void_p), len(buf),
                                 ctypes.byref(h), ctypes.byref(w), ctypes.byref(c)),
               "idn_jpeg_info")
    if not orientation and jpeg_orientation(buf) >= 5:  # back to the decoded (untransposed) size
        return w.value, h.value, c.value
    return h.value, w.value, c.value


JPEG_MODES = {"libjpeg9": 0, "turbo": 1}  # include/idn.h IDN_JPEG_TURBO
JPEG_IGNORE_ORIENTATION = 2  # include/idn.h IDN_JPEG_IGNORE_ORIENTATION


def jpeg_decode(files, out: Optional[torch.Tensor] = None, device=None, mode: str = "libjpeg9",
                chunk_bits: int = 0, orientation: bool = True) -> torch.Tensor:
    """cv2.imread(path) for a batch of same-size JPEG files (bytes in host memory):
    (n, h, w, 3) uint8 BGR on the GPU.  mode "libjpeg9" (default) is bit-exact with the
    reference's pinned IJG libjpeg 9d (requirements.txt:74, under OpenCV 3.4.2: scaled 16x16 /
    16x8 chroma IDCT); "turbo" with libjpeg-turbo (fancy upsampling).  Each image is turned by its
    EXIF orientation as OpenCV 3.4.2's imread does (orientation=False: cv2's
    IMREAD_IGNORE_ORIENTATION); (h, w) is the size after the turn and must agree across the
    batch.  chunk_bits (0 = default) sets the entropy decoder's chunk size; it does not change
    the output."""
    files = list(files)
    if not files:
        raise ValueError("jpeg_decode: no files")
    if mode not in JPEG_MODES:
        raise ValueError(f"jpeg_decode: mode must be one of {sorted(JPEG_MODES)}")
    flags = JPEG_MODES[mode] | (int(chunk_bits) << 8) | (0 if orientation else JPEG_IGNORE_ORIENTATION)
    h, w, _ = jpeg_info(files[0], orientation)
    n = len(files)
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if out is None:
        out = torch.empty((n, h, w, 3), dtype=torch.uint8, device=dev)
    elif (out.dtype != torch.uint8 or tuple(out.shape) != (n, h, w, 3) or not out.is_contiguous()
          or out.device.type != "cuda"):
        raise ValueError("jpeg_decode: out must be a contiguous (n, h, w, 3) uint8 CUDA tensor")
    lib = _lib.load()
    bufs, ptrs, lens = _file_ptrs(files)
    ws_bytes = lib.idn_jpeg_workspace_size(ptrs, lens, n, flags)
    if ws_bytes == 0:
        raise _lib.IdnError("jpeg_decode: unsupported or corrupt JPEG in the batch (or bad flags)")
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=out.device)
    with torch.cuda.device(out.device):
        rc = lib.idn_jpeg_decode_u8(ptrs, lens, n, out.data_ptr(), h, w, w * 3, flags,
                                    ws.data_ptr(), ws_bytes, _stream())
    _lib.check(rc, "idn_jpeg_decode_u8")
    del bufs
    return out
