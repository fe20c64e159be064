#!/usr/bin/env python3
"""Headline benchmark: Mpix/s filtered by the 5x5 GaussianBlur (cv2.GaussianBlur(u8,(5,5),0)
semantics, bit-exact) on synthetic 600x1000x3 uint8 images resident in HBM.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--op gauss5|gauss3|box3|...]

One step = one pass of the filter over one batch of B images (default 256, BASELINE config 2's
batch with the metric's 5x5 Gaussian).  For N > 1 the driver launches one process per GPU
(torch.distributed.run); each rank owns its own B-image shard (weak scaling, images are
independent: no collective in the timed region), the timed region is bracketed by
barrier + synchronize and the max over ranks is reported.  Rank 0 prints ONE JSON line with the
roofline object of the dominant kernel (algorithmic 6 B/pixel over the HIP-event-timed launch
duration) and the CPU baseline (oracle C restatement of the same filter, OpenMP, bounded sample).
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "image-denoising_amd"))
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
H, W, C = 600, 1000, 3

OPS = {
    # name: (metric label, idn call, algorithmic bytes per pixel, kernel name prefix)
    "gauss5": ("5x5 Gaussian", lambda idn, x, y: idn.gaussian_blur(x, 5, out=y), 6, "stencil_u8"),
    "gauss3": ("3x3 Gaussian", lambda idn, x, y: idn.gaussian_blur(x, 3, out=y), 6, "stencil_u8"),
    "box3": ("3x3 mean", lambda idn, x, y: idn.blur(x, 3, out=y), 6, "stencil_u8"),
    "median5": ("5x5 median", lambda idn, x, y: idn.median_blur(x, 5, out=y), 6, "median_u8"),
    "median3": ("3x3 median", lambda idn, x, y: idn.median_blur(x, 3, out=y), 6, "median_u8"),
    "bilateral": ("bilateral d=9 s=75/75",
                  lambda idn, x, y: idn.bilateral_filter(x, 9, 75.0, 75.0, out=y), 6, "bilateral_u8"),
    # skimage random_noise('gaussian', var=1.0) + U8 cast, Philox stream (BASELINE config 2 noise)
    "noise_gaussian": ("gaussian_var1.0 noise",
                       lambda idn, x, y: idn.ops.random_noise(x, "gaussian", var=1.0, seed=3, out="u8",
                                                              out_u8=y), 6, "noise_gauss"),
    # skimage random_noise('s&p', amount=0.4) + U8 cast, Philox stream (BASELINE config 3 noise)
    "noise_sap": ("sap_var0.4 noise",
                  lambda idn, x, y: idn.ops.random_noise(x, "s&p", amount=0.4, seed=3, out="u8",
                                                         out_u8=y), 6, "noise_flat16"),
    # skimage random_noise('poisson') + U8 cast, Philox stream (BASELINE config 5 noise type)
    "noise_poisson": ("poisson noise",
                      lambda idn, x, y: idn.ops.random_noise(x, "poisson", seed=3, out="u8",
                                                             out_u8=y), 6, "noise_poisson"),
    # 3-level Haar BayesShrink soft threshold (BASELINE config 5 denoiser), fp64 pipeline
    "wavelet_haar3": ("3-level Haar wavelet",
                      lambda idn, x, y: idn.ops.denoise_wavelet(x, "db1", 3, out_u8=y), 6, "wl_"),
    # bior1.5, default levels (the reference's live denoiser: test.py:1807-1810)
    "wavelet_bior15": ("bior1.5 wavelet (default levels)",
                       lambda idn, x, y: idn.ops.denoise_wavelet(x, "bior1.5", None, out_u8=y), 6,
                       "wl_"),
    # 5x5 Gaussian straight into the float32 blob (3 B read + 12 B written per pixel)
    "gauss5_blob": ("5x5 Gaussian -> f32 blob", None, 15, "stencil_u8"),
    # quant noise, k = 7 (MiniBatchKMeans colour quantisation in Lab: fit + apply)
    "quant7": ("quant k=7", lambda idn, x, y: idn.ops.quantize(x, 7, seed=3, out=y), 6, "quant_"),
}
# arithmetic type each op computes in (the filters are integer SWAR / fixed point)
# (the Philox u8 noise streams: fp32 Box-Muller on 16-bit uniforms, fp32 apply on the 0..255
# scale; s&p integer thresholds on 16-bit uniforms; Poisson integer CDF thresholds)
_U8NOISE = "f32 apply, 16-bit-uniform Box-Muller (32-bit tail refinement)"
DTYPE = {"noise_gaussian": _U8NOISE, "noise_sap": "u32 (16-bit uniform thresholds)",
         "noise_poisson": "u32 (CDF thresholds)", "wavelet_haar3": "f64", "bilateral": "f32",
         "cfg2": _U8NOISE + " + u16 SWAR filter", "cfg2p": _U8NOISE + " + u16 SWAR filter",
         "wavelet_bior15": "f64 normalisation / finest-dd / sums of squares, f32 lowpass and "
                           "synthesis", "gauss5_blob": "u8->f32", "quant7": "i32/f64",
         "cfg3": "u32 noise + f16-lane median", "cfg4": _U8NOISE + " + f32 bilateral",
         "cfg5": "f32/u32 noise + f64 wavelet", "jpeg_decode": "i32 (integer IDCT)"}
PARITY = {"noise_gaussian": "skimage random_noise('gaussian') U8 law (chi-square tested at the "
                            "reference's levels; bit-exact under replay)",
          "noise_poisson": "skimage random_noise('poisson') law (bit-exact under replay)",
          "noise_sap": "skimage random_noise('s&p') law (bit-exact under replay)",
          "wavelet_haar3": "skimage 0.14 denoise_wavelet within 1e-5",
          "bilateral": "cv2.bilateralFilter within 1 LSB",
          "cfg2": "Philox noise + cv2.blur bit-exact", "cfg3": "Philox s&p + cv2.medianBlur bit-exact",
"cfg2p": "Philox noise + cv2.blur bit-exact",
          "wavelet_bior15": "skimage 0.14 denoise_wavelet within 1e-5",
          "gauss5_blob": "cv2.GaussianBlur + blob.py float32 LUT, bit-exact",
          "quant7": "OpenCV 8-bit Lab + k-means (sklearn-replay bit-exact; device fit within 5% "
                    "inertia)",
          "cfg4": "Philox speckle + cv2.bilateralFilter within 1 LSB",
          "cfg5": "Philox/periodic noise + denoise_wavelet within 1e-5",
          "jpeg_decode": "IJG libjpeg 9d decode (ISLOW + scaled 16x16 chroma IDCT), bit-exact vs "
                         "the reference's pinned library"}
# ops that synchronise inside the call (host work, H2D copies, convergence polls): their event
# time is the op's end-to-end duration, not a kernel's, so no HBM fraction is claimed for them
END_TO_END = {"jpeg_decode", "detect_e2e", "detect_e2e_pipelined"}

def _pipeline(kind):
    """BASELINE.json configs 2-5 as one step = noise + denoise over the batch (intermediate u8
    buffers are allocated once, outside the timed region)."""
    state = {}

    def step(idn, x, y):
        import torch
        t = state.get("t")
        if t is None or t.shape != x.shape:
            t = state["t"] = x.new_empty(x.shape)
        ops = idn.ops
        if kind == "cfg2":    # gaussian_var1.0 + mean 3x3: noise launch, then the filter
            ops.random_noise(x, "gaussian", var=1.0, seed=3, out="u8", out_u8=t)
            idn.blur(t, 3, out=y)
        elif kind == "cfg2p":  # chunked: noise of chunk k+1 beside the filter of chunk k
            ops.noise_filter(x, "gaussian", "mean", 3, var=1.0, seed=3, out=y, form="pipelined")
        elif kind == "cfg3":  # sap_var0.4 + median 5x5
            ops.random_noise(x, "s&p", amount=0.4, seed=3, out="u8", out_u8=t)
            idn.median_blur(t, 5, out=y)
        elif kind == "cfg4":  # speckle_var1.0 + bilateral d=9 sigma 75/75
            ops.random_noise(x, "speckle", var=1.0, seed=3, out="u8", out_u8=t)
            idn.bilateral_filter(t, 9, 75.0, 75.0, out=y)
        else:                 # cfg5: mixed noise (one type per image, seeded) + Haar L=3 wavelet
            groups = state.get("groups")
            if groups is None:
                import random
                rng = random.Random(3)
                kinds = [rng.choice(["gaussian", "s&p", "speckle", "poisson", "periodic",
                                     "original"]) for _ in range(x.shape[0])]
                groups = {}
                for i, k in enumerate(kinds):
                    groups.setdefault(k, []).append(i)
                # images of a type are scattered through the batch, as a mixed loader yields them:
                # each type is noised in place in the full batch (its batch positions as slots,
                # its image ids for the streams) in one launch -- no gather / scatter
                state["groups"] = groups = {
                    k: (v, torch.as_tensor(v, dtype=torch.int64, device=x.device))
                    for k, v in groups.items()}
            for k, (_, idx) in groups.items():
                if k == "original":
                    ops.copy_slots(x, t, idx)
                elif k == "periodic":
                    ops.periodic_noise(x, 100.0, out=t, slots=idx)
                elif k == "s&p":
                    ops.random_noise(x, "s&p", amount=0.4, seed=3, image_ids=idx, slots=idx,
                                     out_u8=t)
                elif k == "poisson":
                    ops.random_noise(x, "poisson", seed=3, image_ids=idx, slots=idx, out_u8=t)
                else:
                    ops.random_noise(x, k, var=1.0, seed=3, image_ids=idx, slots=idx, out_u8=t)
            ops.denoise_wavelet(t, "db1", 3, out_u8=y)
    step.state = state
    return step


PIPELINES = {
    "cfg2": ("gaussian_var1.0 + 3x3 mean (config 2)", 256),
    "cfg2p": ("gaussian_var1.0 + 3x3 mean (config 2, chunk-pipelined on two streams)", 256),
    "cfg3": ("sap_var0.4 + 5x5 median (config 3)", 1024),
    "cfg4": ("speckle_var1.0 + bilateral d=9 s=75/75 (config 4)", 512),
    "cfg5": ("mixed noise + 3-level Haar wavelet (config 5)", 512),
}
for _k, (_lbl, _b) in PIPELINES.items():
    OPS[_k] = (_lbl, _pipeline(_k), 6, "pipeline")


def _gauss5_blob(idn, x, y):
    st = _gauss5_blob.__dict__
    b = st.get("blob")
    if b is None or b.shape != x.shape:
        import torch
        b = st["blob"] = torch.empty(x.shape, dtype=torch.float32, device=x.device)
    idn.ops.gaussian_blob(x, 5, out=b)


OPS["gauss5_blob"] = (OPS["gauss5_blob"][0], _gauss5_blob, 15, "stencil_u8")


def _wavelet_bior15_f64(idn, x, y):
    """the live test path's denoiser input: random_noise's float64 image (lib/model/test.py:1678-1684
    -> 1807-1810); the f64 copy (img_as_float of the batch) is made once, untimed"""
    st = _wavelet_bior15_f64.__dict__
    f = st.get("f64")
    if f is None or f.shape != x.shape:
        f = st["f64"] = x.double() * (1.0 / 255.0)
    idn.ops.denoise_wavelet(f, "bior1.5", None, out_u8=y)


# 24 B of float64 read + 3 B written per pixel
OPS["wavelet_bior15_f64"] = ("bior1.5 wavelet on float64 input (live test path)", _wavelet_bior15_f64,
                             27, "wl_")
DTYPE["wavelet_bior15_f64"] = DTYPE["wavelet_bior15"]
PARITY["wavelet_bior15_f64"] = PARITY["wavelet_bior15"]


def _live_f64(fused):
    """the live test path's noise + denoise on the batch (lib/model/test.py:1678-1684 ->
    1802-1810): random_noise(gaussian, var 0.1) as float64, then denoise_wavelet(bior1.5) on that
    float64 image; fused = the noise kernel reduces the wavelet's colour range as it writes the
    image (random_noise_ycc -> denoise_wavelet(ycc_keys)), else the two plain calls"""
    def step(idn, x, y):
        if fused:
            f, keys = idn.ops.random_noise_ycc(x, "gaussian", var=0.1, seed=3)
            idn.ops.denoise_wavelet(f, "bior1.5", None, out_u8=y, ycc_keys=keys)
        else:
            f = idn.ops.random_noise(x, "gaussian", var=0.1, seed=3, out="f64")
            idn.ops.denoise_wavelet(f, "bior1.5", None, out_u8=y)
    return step


# 3 B read + 24 B (f64) written by the noise, 24 B read + 3 B written by the wavelet per pixel
OPS["live_f64"] = ("gaussian_var0.1 (float64) + bior1.5 wavelet, fused colour range (live test "
                   "path)", _live_f64(True), 54, "pipeline")
OPS["live_f64_unfused"] = ("gaussian_var0.1 (float64) + bior1.5 wavelet, two plain calls",
                           _live_f64(False), 54, "pipeline")
for _k in ("live_f64", "live_f64_unfused"):
    DTYPE[_k] = "f64 noise + " + DTYPE["wavelet_bior15"]
    PARITY[_k] = "Philox f64 gaussian law + skimage 0.14 denoise_wavelet within 1e-5"


def _jpeg_files(x, quality=90):
    """the batch encoded once (untimed) by Pillow: baseline 4:2:0 JPEG files in host memory"""
    import io
    from PIL import Image
    arr = x.cpu().numpy()
    out = []
    for im in arr:
        b = io.BytesIO()
        Image.fromarray(im[..., ::-1]).save(b, "JPEG", quality=quality, subsampling=2)
        out.append(b.getvalue())
    return out


def _jpeg_decode(idn, x, y):
    st = _jpeg_decode.__dict__
    if st.get("n") != x.shape[0]:
        st["files"] = _jpeg_files(x)
        st["n"] = x.shape[0]
    idn.ops.jpeg_decode(st["files"], out=y)


# cv2.imread of the batch's JPEG files (host memory -> one H2D copy -> GPU decode), q90 4:2:0
OPS["jpeg_decode"] = ("JPEG decode (cv2.imread), q90 4:2:0 files in host memory", _jpeg_decode, 3,
                      "jpeg_")

def _detect_e2e(idn, x, y):
    """The reference's per-image test loop body as one step (lib/model/test.py:189-191,
    1678-1684, 1787-1811, 85-90): a 600x1000 q90 4:2:0 JPEG file on disk -> GPU decode
    (cv2.imread) -> apply_noise('gaussian_wavelet_var0.1', test_v0: random gaussian level, float64
    plain branch, the live bior1.5 wavelet hook) -> _get_blobs -> the float32 blob in host memory
    (numpy), as net.test_image is fed.  Batch 1 (IMS_PER_BATCH = 1): the figure is latency."""
    st = _detect_e2e.__dict__
    if "path" not in st:
        import tempfile
        from PIL import Image
        d = tempfile.mkdtemp(prefix="idn_bench_")
        st["path"] = os.path.join(d, "im.jpg")
        Image.fromarray(x[0].cpu().numpy()[..., ::-1]).save(st["path"], "JPEG", quality=90,
                                                             subsampling=2)
    from idn import detect_blob
    im = detect_blob.apply_noise(st["path"], "gaussian_wavelet_var0.1", mode="test_v0",
                                 decode="gpu", as_tensor=True)
    detect_blob._get_blobs(im)


OPS["detect_e2e"] = ("per-image test_net body: JPEG -> gaussian_wavelet (test_v0) -> blob, numpy out",
                     _detect_e2e, 6, "e2e")


def _detect_e2e_pipelined(idn, x, y):
    """The same body over the reference's image loop (test.py:189-191) with idn.io.ImageReader:
    the files are decoded in windows of 8 (one launch each), window b + 1 on a side stream while
    the images of window b go through noise, wavelet, blob and the host copy.
    Eight distinct 600x1000 q90 files in turn; a step is one image of the loop."""
    st = _detect_e2e_pipelined.__dict__
    if "paths" not in st:
        import tempfile
        from PIL import Image
        d = tempfile.mkdtemp(prefix="idn_bench_")
        st["paths"] = []
        for j in range(8):
            p = os.path.join(d, f"im{j}.jpg")
            import numpy as np
            im = x[0].cpu().numpy()[..., ::-1]
            Image.fromarray(np.ascontiguousarray(np.roll(im, 37 * j, axis=1))).save(
                p, "JPEG", quality=90, subsampling=2)
            st["paths"].append(p)
        st["k"] = 0
        from idn import io as idn_io
        st["reader"] = idn_io.ImageReader(st["paths"] * 100000,
                                          batch=int(os.environ.get("IDN_BENCH_READ_BATCH", "8")))
    from idn import detect_blob
    im = detect_blob.apply_noise(st["reader"][st["k"]], "gaussian_wavelet_var0.1", mode="test_v0",
                                 decode="gpu", as_tensor=True)
    detect_blob._get_blobs(im)
    st["k"] += 1


OPS["detect_e2e_pipelined"] = ("per-image test_net loop: JPEG -> gaussian_wavelet (test_v0) -> "
                               "blob, numpy out; files decoded 8 at a time, the next window ahead (idn.io.ImageReader)",
                               _detect_e2e_pipelined, 6, "e2e")

METRIC = "Mpix/s filtered (5\u00d75 Gaussian, 1000\u00d7600) at 1/2/4/8 GPUs; % HBM roofline"


def synth_batch(torch, n, dev, seed=3):
    """On-device textured pattern: clip(128 + 64 sin(2πx/97) cos(2πy/61)
    + U(-32,32), 0, 255) per channel, uint8."""
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    y = torch.arange(H, device=dev, dtype=torch.float32).view(1, H, 1, 1)
    x = torch.arange(W, device=dev, dtype=torch.float32).view(1, 1, W, 1)
    base = 128 + 64 * torch.sin(2 * torch.pi * x / 97) * torch.cos(2 * torch.pi * y / 61)
    out = torch.empty((n, H, W, C), dtype=torch.uint8, device=dev)
    for i in range(0, n, 64):
        m = min(64, n - i)
        u = torch.rand((m, H, W, C), generator=g, device=dev) * 64 - 32
        out[i:i + m] = (base + u).clamp_(0, 255).to(torch.uint8)
    return out


def cpu_baseline(op: str, budget_s: float = 12.0):
    """Oracle C restatement (OpenMP) of the same filter on the host, bounded sample."""
    import numpy as np
    import oracle
    sys.path.insert(0, str(ROOT / "tests"))
    table = {
        "gauss5": lambda a: oracle.cv.gaussian_blur_fast(a, 5),
        "gauss3": lambda a: oracle.cv.gaussian_blur_fast(a, 3),
        "box3": lambda a: oracle.cv.blur(a, 3),
        "median5": lambda a: oracle.cv.median_blur(a, 5),
        "median3": lambda a: oracle.cv.median_blur(a, 3),
        "bilateral": lambda a: oracle.cv.bilateral_filter(a, 9, 75.0, 75.0),
        "noise_gaussian": lambda a: oracle.sk.to_u8(255 * oracle.sk.noise_gaussian(
            a, np.random.normal(0.0, 1.0, a.shape))),
        "noise_sap": lambda a: oracle.sk.to_u8(255 * oracle.sk.noise_sap(
            a, np.random.random_sample(a.shape), np.random.random_sample(a.shape), 0.4)),
        "noise_poisson": lambda a: oracle.sk.to_u8(255 * oracle.sk.noise_poisson(
            a[0], np.random.poisson(oracle.sk.poisson_lambda(a[0])))),
        "wavelet_haar3": lambda a: oracle.sk.to_u8(255 * oracle.wavelet.denoise_wavelet(a[0], "db1", 3)),
        "cfg2": lambda a: oracle.cv.blur(oracle.sk.to_u8(255 * oracle.sk.noise_gaussian(
            a, np.random.normal(0.0, 1.0, a.shape))), 3),
        "cfg3": lambda a: oracle.cv.median_blur(oracle.sk.to_u8(255 * oracle.sk.noise_sap(
            a, np.random.random_sample(a.shape), np.random.random_sample(a.shape), 0.4)), 5),
        "cfg4": lambda a: oracle.cv.bilateral_filter(oracle.sk.to_u8(255 * oracle.sk.noise_speckle(
            a, np.random.normal(0.0, 1.0, a.shape))), 9, 75.0, 75.0),
        "cfg5": lambda a: oracle.sk.to_u8(255 * oracle.wavelet.denoise_wavelet(oracle.sk.to_u8(
            255 * oracle.sk.noise_gaussian(a[0], np.random.normal(0.0, 1.0, a[0].shape))), "db1", 3)),
        "wavelet_bior15": lambda a: oracle.sk.to_u8(
            255 * oracle.wavelet.denoise_wavelet(a[0], "bior1.5", None)),
        "wavelet_bior15_f64": lambda a: oracle.sk.to_u8(
            255 * oracle.wavelet.denoise_wavelet(a[0] * (1.0 / 255.0), "bior1.5", None)),
        "gauss5_blob": lambda a: oracle.sk.blob_f32(oracle.cv.gaussian_blur_fast(a, 5)),
        # the per-image body on the host: decode, f64 gaussian noise, bior1.5 wavelet, blob
        "detect_e2e": lambda a: oracle.sk.blob_f32([oracle.wavelet.denoise_wavelet(
            oracle.sk.noise_gaussian(a[0], np.random.normal(0.0, 1.0, a[0].shape)),
            "bior1.5", None)]),  # test_v0 quirk: the float64 [0, 1] image goes to the blob
    }
    table["cfg2p"] = table["cfg2"]
    table["detect_e2e_pipelined"] = table["detect_e2e"]
    table["live_f64"] = table["live_f64_unfused"] = lambda a: oracle.sk.to_u8(
        255 * oracle.wavelet.denoise_wavelet(oracle.sk.noise_gaussian(
            a[0], np.random.normal(0.0, 0.1 ** 0.5, a[0].shape)), "bior1.5", None))
    if op == "jpeg_decode":  # Pillow's libjpeg-turbo decode of the same kind of file
        import io
        from PIL import Image
        rs0 = np.random.RandomState(3)
        src = np.clip(128 + rs0.uniform(-64, 64, size=(H, W, C)), 0, 255).astype(np.uint8)
        bio = io.BytesIO()
        Image.fromarray(src).save(bio, "JPEG", quality=90, subsampling=2)
        data = bio.getvalue()

        def _pil(a):
            with Image.open(io.BytesIO(data)) as im:
                return np.asarray(im.convert("RGB"))
        table["jpeg_decode"] = _pil
    fn = table.get(op)
    if fn is None:
        return None
    rs = np.random.RandomState(3)
    nb = 16 if op in ("gauss5", "gauss3", "gauss5_blob") else 1  # threaded: a batch per call
    img = np.clip(128 + rs.uniform(-64, 64, size=(nb, H, W, C)), 0, 255).astype(np.uint8)
    fn(img)  # warm (build + page in)
    n_img, t0 = 0, time.perf_counter()
    while True:
        fn(img)
        n_img += nb
        el = time.perf_counter() - t0
        if el >= budget_s or n_img >= 1000000:
            break
    if op in ("noise_gaussian", "noise_sap", "noise_poisson", "wavelet_haar3", "cfg5",
              "wavelet_bior15", "wavelet_bior15_f64", "detect_e2e", "detect_e2e_pipelined", "live_f64",
              "live_f64_unfused"):
        threads, src = 1, "numpy, single thread"
    elif op == "jpeg_decode":
        threads, src = 1, "PIL (libjpeg-turbo) decode, single thread"
    elif op in ("cfg2", "cfg2p", "cfg3", "cfg4"):
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
        src = "numpy noise (1 thread) + oracle/filters.c OpenMP"
    elif op in ("gauss5", "gauss3", "gauss5_blob"):
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
        src = ("oracle/baseline_fast.c: separable 16-bit SIMD (AVX2) + OpenMP, OpenCV's 8-bit "
               "scheme, bit-exact with the scalar oracle")
    else:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
        src = "oracle/filters.c OpenMP"
    return {
        "value": round(n_img * H * W / el / 1e6, 3),
        "unit": "Mpix/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{n_img} x {H}x{W}x3 u8 images, {op}: {src}; {threads} threads, "
                  f"{el:.1f} s; the same {nb}-image batch ({nb * H * W * C / 1e6:.1f} MB) "
                  f"re-filtered each call, so it is cache-resident (a conservative, i.e. "
                  f"favourable-to-CPU, baseline; the GPU line streams its batch from HBM) "
                  f"(restatement -- cv2/skimage are not installed, so the reference's own CPU "
                  f"path cannot run here)",
    }


def load_traffic(op: str):
    """HBM bytes per launch from the committed PMC summary (profiles/pmc_traffic.json), or None.
    Not measured in this run: the counters need their own rocprofv3 --pmc passes."""
    p = ROOT / "profiles" / "pmc_traffic.json"
    if not p.exists():
        return None
    try:
        d = json.loads(p.read_text())
        return d.get(op, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


# VALU issue peak in lane operations per second: 256 CUs x 4 SIMDs x 16 lanes x 2.4 GHz (a wave64
# VALU instruction issues over 4 cycles; fp64 FMA runs at the same per-lane rate on gfx950,
# MI355X_MICROARCH.md), i.e. 39.3 T lane-ops/s -- the binding roofline of the ops whose counters
# show VALU issue near saturation (VALU utilisation beside the %HBM figure)
VALU_PEAK = 256 * 4 * 16 * 2.4e9


def load_valu(op: str):
    """VALU lane operations per pixel of the op (all its kernels) from the newest committed
    rocprofv3 --pmc record profiles/r*/pmc/<op>.json (SQ_INSTS_VALU x 64 / pixels of the launch),
    or None.  Not measured in this run: the SQ counters need their own --pmc passes."""
    recs = sorted(ROOT.glob(f"profiles/r*/pmc/{op}.json"))
    for p in reversed(recs):
        try:
            d = json.loads(p.read_text())
        except Exception:
            continue
        ks = d.get("kernels", {})
        vpp = [k["valu_per_pixel"] for k in ks.values() if k.get("valu_per_pixel") is not None]
        if vpp:
            main = max(ks.items(), key=lambda kv: kv[1].get("avg_us") or 0.0)[0]
            return {"valu_per_pixel": round(sum(vpp), 2), "kernels": len(vpp),
                    "longest_kernel": main, "source": str(p.relative_to(ROOT))}
    return None


def roofline_fields(op, bpp, pixels, avg_kern_ms, traffic, kname):
    """The roofline object: the HBM roofline (algorithmic bytes / the line's kernel time) and,
    where a committed PMC record gives the op's VALU lane-ops per pixel, the VALU roofline over
    the same time; `bound` is whichever fraction is higher and the top-level achieved / peak /
    unit / frac are that roofline's."""
    achieved_gbs = bpp * pixels / (avg_kern_ms * 1e-3) / 1e9
    e2e = op in END_TO_END
    hbm = {"achieved": round(achieved_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": None if e2e else round(achieved_gbs / HBM_PEAK_GBS, 4)}
    rl = {"bound": "latency (end-to-end op)" if e2e else "hbm", **hbm, "hbm": dict(hbm),
          "traffic": traffic,
          "traffic_source": "profiles/pmc_traffic.json (committed rocprofv3 FETCH_SIZE x2 + "
                            "WRITE_SIZE passes; not measured in this run)" if traffic else None}
    v = None if e2e else load_valu(op)
    if v is not None:
        lane_ops = v["valu_per_pixel"] * pixels / (avg_kern_ms * 1e-3)
        rl["valu"] = {"achieved": round(lane_ops / 1e12, 3), "peak": round(VALU_PEAK / 1e12, 3),
                      "unit": "T lane-ops/s", "frac": round(lane_ops / VALU_PEAK, 4),
                      "valu_per_pixel": v["valu_per_pixel"],
                      "valu_source": v["source"] + " (SQ_INSTS_VALU x 64 / pixels; counters "
                                                   "not measured in this run)"}
        if rl["valu"]["frac"] > hbm["frac"]:
            rl.update(bound="valu", achieved=rl["valu"]["achieved"], peak=rl["valu"]["peak"],
                      unit=rl["valu"]["unit"], frac=rl["valu"]["frac"])
    rl.update({"kernel": kname, "kernel_ms_avg": round(avg_kern_ms, 5)})
    return rl, achieved_gbs


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` outside torchrun: start the N ranks as ONE child process group
    (python -m torch.distributed.run, one process per GPU) before anything touches the GPU, pass
    rank 0's JSON line through, and return the child's exit code."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           str(Path(__file__).resolve()), *sys.argv[1:]]
    return subprocess.run(cmd, env=env).returncode


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=0, help="images per GPU (weak scaling; default "
                    "256, or the config's per-GPU batch for cfg2..cfg5) or in total (strong)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak",
                    help="weak: every rank filters --batch images; strong: --batch images in "
                         "total, split into contiguous shards over the ranks")
    ap.add_argument("--op", default="gauss5", choices=sorted(OPS))
    ap.add_argument("--settle-s", type=float, default=0.5,
                    help="after the W warmup steps, keep stepping (untimed) until this many seconds "
                         "of sustained load have passed: the GPU's power controller settles the "
                         "clocks of a power-capped kernel over the first ~30-50 ms "
                         "(profiles/r02/clock/), and the timed K steps should see that steady state")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-copy", action="store_true", help="skip the same-run copy ceiling")
    ap.add_argument("--gather", action="store_true",
                    help="N>1: also time reassembling the filtered batch on every rank with one "
                         "RCCL all-gather over xGMI per step (reported as 'allgather')")
    ap.add_argument("--lib", choices=("product", "tuning"), default="product",
                    help="tools only: run through the tuning build (knobs from the environment)")
    ap.add_argument("--dry-run", action="store_true",
                    help="resolve ranks and shards and print them without touching a GPU (tests)")
    return ap.parse_args(argv)


def copy_ceiling(idn, torch, x, y, reps: int = 20):
    """Same-run copy ceiling over the op's own buffers (x -> y, x.nbytes read + written): the
    flat burst copy at default and nontemporal policy, HIP events over `reps` launches each."""
    out = {}
    for pol, name in ((0, "default"), (1, "nontemporal")):
        for _ in range(3):
            idn.ops.copy_flat(x, y, pol)
        st = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            idn.ops.copy_flat(x, y, pol)
        e1.record(st)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / reps
        out[name] = round(2 * x.nbytes / (ms * 1e-3) / 1e9, 1)
    return {"copy_ceiling_GBps": max(out.values()), "by_policy": out,
            "bytes_per_launch": 2 * x.nbytes, "kernel": "copy_burst_kernel"}


def main():
    args = parse_args()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(world_env or "1")
    if args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch N ranks with "
              f"torch.distributed.run --nproc-per-node {args.gpus} (or drop WORLD_SIZE and let "
              f"bench.py start them)", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.batch <= 0:
        args.batch = (PIPELINES[args.op][1] if args.op in PIPELINES else
                      1 if args.op in ("detect_e2e", "detect_e2e_pipelined") else 256)
    if args.scaling == "strong":
        from idn.parallel import shard_range
        lo, hi = shard_range(args.batch, rank, world)
        total_images = args.batch
    else:
        lo, hi = rank * args.batch, (rank + 1) * args.batch
        total_images = args.batch * world
    my_batch = hi - lo
    if args.dry_run:
        import torch.distributed as dist
        if world > 1:
            dist.init_process_group("gloo")
            got = [None] * world
            dist.all_gather_object(got, [rank, lo, hi])
            dist.destroy_process_group()
        else:
            got = [[0, lo, hi]]
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "scaling": args.scaling,
                              "total_images": total_images, "shards": got}), flush=True)
        return

    import torch
    import torch.distributed as dist
    import idn

    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    tuning = contextlib.ExitStack()
    if args.lib == "tuning":  # A/B runs of the kernels' tuning knobs (never the driver's line)
        from idn import _lib
        # held open for the whole run (a bare variant(...).__enter__() on a temporary reverts
        # as soon as the context manager is collected)
        tuning.enter_context(_lib.variant("tuning"))
    label, call, bpp, kname = OPS[args.op]
    x = synth_batch(torch, my_batch, dev, seed=3 + rank)
    y = torch.empty_like(x)
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        call(idn, x, y)
    torch.cuda.synchronize()
    # sustained-load settle (untimed): chunks of launches until settle_s seconds have passed
    settle_steps, ts0 = 0, time.perf_counter()
    while time.perf_counter() - ts0 < args.settle_s:
        for _ in range(16):
            call(idn, x, y)
        settle_steps += 16
        torch.cuda.synchronize()
    settle_s = time.perf_counter() - ts0

    stream = torch.cuda.current_stream()
    # kernel time: one HIP event pair around the K back-to-back launches on the launch stream
    # (region / K); event pairs around every launch add their own dispatch gaps (~2-4 us, a few
    # % of a 0.17 ms kernel) -- those are kept for the median only
    e_beg, e_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e_beg.record(stream)
    for i in range(args.steps):
        call(idn, x, y)
    e_end.record(stream)
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    wall = t1 - t0
    avg_kern_ms = e_beg.elapsed_time(e_end) / args.steps
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(min(args.steps, 10))]
    for a, b in ev:  # untimed by the wall clock: per-launch pairs for the median
        a.record(stream)
        call(idn, x, y)
        b.record(stream)
    torch.cuda.synchronize()
    kern_ms = sorted(a.elapsed_time(b) for a, b in ev)

    if world > 1:
        t = torch.tensor([wall], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())

    gather = None
    if world > 1 and args.gather:
        # end-to-end figure = filter step + all-gather of every rank's u8 output
        from idn.parallel import all_gather_batch
        full =torch.empty((world * my_batch, H, W, C), dtype=torch.uint8, device=dev)
        gather_once = ((lambda: all_gather_batch(y, total_images)) if args.scaling == "strong"
                       else (lambda: dist.all_gather_into_tensor(full, y)))
        for _ in range(2):
            gather_once()
        torch.cuda.synchronize()
        barrier()
        g0 = time.perf_counter()
        for _ in range(args.steps):
            gather_once()
        torch.cuda.synchronize()
        barrier()
        gt = torch.tensor([time.perf_counter() - g0], device=dev, dtype=torch.float64)
        dist.all_reduce(gt, op=dist.ReduceOp.MAX)
        g_ms = float(gt.item()) / args.steps * 1e3
        del full
        gather = {"ms_per_step": round(g_ms, 4), "bytes_per_rank": int(y.numel()),
                  "algbw_GBps": round(y.numel() * (world - 1) / (g_ms * 1e-3) / 1e9, 1)}

    ceiling = None
    if not args.no_copy and rank == 0:
        ceiling = copy_ceiling(idn, torch, x, y)

    pix_step = total_images * H * W
    value = pix_step * args.steps / wall / 1e6
    traffic = load_traffic(args.op)
    roofline, achieved_gbs = roofline_fields(args.op, bpp, my_batch * H * W, avg_kern_ms, traffic,
                                             kname)

    if rank == 0:
        rec = {
            "metric": METRIC if args.op == "gauss5" else
                      f"Mpix/s filtered ({label}, 1000x600) at 1/2/4/8 GPUs; % HBM roofline",
            "value": round(value, 1),
            "unit": "Mpix/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle": {"seconds": round(settle_s, 3), "steps": settle_steps,
                       "why": "untimed sustained load after the warmup steps so the timed steps "
                              "run at the power controller's steady-state clocks (the first "
                              "~30-50 ms of load swing 160-200 us per launch; see "
                              "profiles/r02/clock/README.md)"},
            "ms_per_step": round(wall / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": DTYPE.get(args.op, "u8"),
            "data": "synthetic (on-device textured pattern, seed 3+rank)",
            "config": {
                "workload": f"{label}, batch {my_batch}x600x1000x3 uint8 per GPU "
                            f"({total_images} in total, {args.scaling} scaling), "
                            + PARITY.get(args.op, "cv2 semantics bit-exact"),
                "op": args.op,
                "batch_per_gpu": my_batch,
                "total_images": total_images,
                "image": [H, W, C],
                "parallelism": f"image-sharded x{world} (no collective in the timed region)",
            },
            "roofline": {
                **roofline,
                "timing": ("end-to-end op time (host gather, H2D, synchronous passes), not a "
                           "kernel duration" if args.op in END_TO_END else
                           "HIP events around the K launches on the launch stream"),
                "kernel_ms_median_event_pairs": round(kern_ms[len(kern_ms) // 2], 5),
                "algorithmic_bytes_per_launch": bpp * my_batch * H * W,
            },
            "cpu_baseline": None if (args.no_cpu or world > 1) else cpu_baseline(args.op),
        }
        if ceiling is not None:
            rec["copy_ceiling_GBps"] = ceiling["copy_ceiling_GBps"]
            rec["roofline"]["frac_of_copy_ceiling"] = round(
                achieved_gbs / ceiling["copy_ceiling_GBps"], 4)
            # the stencil's own cache policy (default loads / stores) against the same-policy copy
            rec["roofline"]["frac_of_default_policy_copy"] = round(
                achieved_gbs / ceiling["by_policy"]["default"], 4)
            rec["copy_ceiling"] = ceiling
        if args.op in ("detect_e2e", "detect_e2e_pipelined"):  # the user-visible number
            rec["ms_per_image"] = round(wall / args.steps * 1e3 / my_batch, 3)
            rec["reference_ms_per_image"] = "65-180 (skimage random_noise / denoise_wavelet on "\
                                            "the host, BASELINE.md)"
        if args.op == "cfg5":  # the drawn noise mix (record it in the output)
            rec["config"]["mix"] = {k: len(v[0]) for k, v in call.state["groups"].items()}
        if gather is not None:
            step_ms = wall / args.steps * 1e3
            gather["e2e_value"] = round(pix_step / ((step_ms + gather["ms_per_step"]) * 1e-3) / 1e6, 1)
            rec["allgather"] = gather
        print(json.dumps(rec), flush=True)

    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
