"""Test helper: execute an idn.noise_spec Plan with the ORACLE's CPU ops, drawing the random fields
from numpy's global RandomState in the order skimage.random_noise does (same as the product's
noise_rng='numpy' mode), so a GPU run and this run see identical noise."""
from __future__ import annotations

import numpy as np

import oracle
from oracle import sk


def _noise(img, step, nxt, rng, quant=None):
    op = step.op
    if op == "original":
        return img
    if op == "quant":
        # the device k-means is seeded by Philox, not numpy: the caller supplies the fitted
        # centres' result (checked against oracle.cvlab.quantize_apply by the caller)
        if quant is None:
            raise ValueError("run_plan: a quant step needs the quant callback")
        return quant(img, int(step.args[0]))
    if op == "periodic":
        from idn import noise_spec as ns
        h, w, c = img.shape
        amp = ns.periodic_amplitude(step.args[0], h * w * c)
        return sk.add_saturate(img, sk.periodic_pattern(h, w, c, amp))
    if op == "shader":
        return oracle.automold.shader(img, 3.0)
    if op == "bloom":
        return oracle.automold.add_sun_flare(img, rng)
    if op in ("gaussian", "speckle"):
        field = np.random.normal(0.0, step.args[0] ** 0.5, img.shape)
        return (sk.noise_gaussian if op == "gaussian" else sk.noise_speckle)(img, field)
    if op == "sap":
        r1 = np.random.random_sample(img.shape)
        r2 = np.random.random_sample(img.shape)
        return sk.noise_sap(img, r1, r2, step.args[0])
    if op == "poisson":
        return sk.noise_poisson(img, np.random.poisson(sk.poisson_lambda(img)))
    level = step.args[0]
    if op == "uniform":
        return sk.noise_uniform(img, np.random.random_sample(img.shape), level)
    if op == "gamma":
        return sk.noise_gamma(img, np.random.standard_gamma(1.99, img.shape), level)
    if op == "rayleigh":
        return sk.noise_rayleigh(img, np.sqrt(np.random.chisquare(2, img.shape)), level)
    if op == "brownian":
        return sk.noise_brownian(img, np.random.normal(size=img.size - 1), level)
    raise ValueError(op)


def _filter(x, step, info=None):
    op, a = step.op, step.args
    if op == "wavelet":
        f = oracle.wavelet.denoise_wavelet(x, a[0], a[1])
        if info is not None:
            info["wavelet_f"] = f  # the float result before the caller's U8 cast
        return sk.to_u8(255 * f), True
    if x.dtype == np.float64:
        if op == "gaus_blur":
            return oracle.cvf.gaussian_blur_f64(x, a[0]), False
        if op == "mean":
            return oracle.cvf.blur_f64(x, a[0]), False
        raise RuntimeError("cv2.error")
    if op == "gaus_blur":
        return oracle.cv.gaussian_blur(x, a[0]), False
    if op == "mean":
        return oracle.cv.blur(x, a[0]), False
    if op == "median":
        return oracle.cv.median_blur(x, a[0]), False
    if op == "bilateral":
        return oracle.cv.bilateral_filter(x, *a), False
    raise ValueError(op)


def run_plan(img: np.ndarray, steps, rng, quant=None, info=None):
    """Returns (output, touched_by_wavelet).  quant(img, k) -> u8 image for a quant step.
    info (a dict) receives 'wavelet_f': the last wavelet step's float result before its cast."""
    cur, wl = img, False
    i = 0
    while i < len(steps):
        st = steps[i]
        nxt = steps[i + 1] if i + 1 < len(steps) else None
        if st.kind == "noise":
            cur = _noise(cur, st, nxt, rng, quant)
        elif st.kind == "cast_u8":
            cur = sk.to_u8(255 * cur)
        else:
            cur, w = _filter(cur, st, info)
            wl = wl or w
        i += 1
    return cur, wl
