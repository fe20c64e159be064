"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by the product path).

numpy restatement of the float64 arithmetic the reference's noise closures, periodic generator
and blob builder perform.  The random fields are INPUTS here (replay): numpy's legacy MT19937
stream cannot be reproduced in parallel, so bit-exact parity is defined given the same field,
and the Philox path is checked statistically (tests/).

  img_as_float      skimage.util.dtype (0.14.2 == 0.18.3: x = v * (1/255) in float64)
  random_noise      skimage.util.noise.random_noise modes gaussian / speckle / s&p / poisson
                    (called at lib/model/test.py:193-590, lib/roi_data_layer/minibatch.py:87-490)
  to_u8             `(255 * out).astype(np.uint8)` (test.py:220-221 etc.): C cast via int32
  periodic_pattern  add_periodic_noise, test.py:1128-1298 / minibatch.py:1034-1206
  blob              lib/utils/blob.py:17-47 (prep_im_for_blob at scale 1.0, im_list_to_blob)

Pinned by tests/golden/*.npz, produced by tests/golden/make_fixtures.py from skimage 0.18.3 /
numpy 1.26.4 (the random_noise algorithm is unchanged since the pinned 0.14.2).
"""
from __future__ import annotations

import numpy as np

PIXEL_MEANS = np.array([[[102.9801, 115.9465, 122.7717]]])  # lib/model/config.py:252


def img_as_float(img: np.ndarray) -> np.ndarray:
    if img.dtype == np.uint8:
        return img.astype(np.float64) * (1.0 / 255.0)
    return img.astype(np.float64, copy=False)


def to_u8(y: np.ndarray) -> np.ndarray:
    """(y).astype(np.uint8) for float64 y as the C cast (uint8)(int32)trunc(y) does it:
    truncate toward zero, wrap mod 256; NaN / |y| >= 2**31 -> 0."""
    y = np.asarray(y, np.float64)
    ok = np.isfinite(y) & (np.abs(y) < 2.0 ** 31)
    t = np.where(ok, np.trunc(np.where(ok, y, 0.0)), 0.0).astype(np.int64)
    return (t & 0xFF).astype(np.uint8)


def noise_gaussian(img, field):
    """random_noise(img, 'gaussian', var) with field = np.random.normal(mean, sqrt(var))."""
    return np.clip(img_as_float(img) + field, 0.0, 1.0)


def noise_speckle(img, field):
    x = img_as_float(img)
    return np.clip(x + x * field, 0.0, 1.0)


def noise_sap(img, r_flip, r_salt, amount, salt_vs_pepper=0.5):
    """s&p: flipped = choice([T,F], p=[p,1-p]) == random_sample < p (whole field first),
    salted likewise with q; out[flipped & salted] = 1, out[flipped & ~salted] = 0."""
    x = img_as_float(img).copy()
    flipped = r_flip < amount
    salted = r_salt < salt_vs_pepper
    x[flipped & salted] = 1.0
    x[flipped & ~salted] = 0.0
    return x


def poisson_vals(img) -> float:
    x = img_as_float(img)
    vals = len(np.unique(x))
    return float(2 ** np.ceil(np.log2(vals)))


def poisson_lambda(img) -> np.ndarray:
    return img_as_float(img) * poisson_vals(img)


def noise_poisson(img, draws):
    """out = clip(Poisson(x*vals) / float(vals), 0, 1) given the integer draws."""
    vals = poisson_vals(img)
    return np.clip(np.asarray(draws, np.float64) / float(vals), 0.0, 1.0)


def periodic_pattern(h: int, w: int, c: int, amplitude: float) -> np.ndarray:
    size = h * w * c
    t = np.linspace(-amplitude, amplitude, size)
    return to_u8(np.sin(t) * 255).reshape(h, w, c)


def add_saturate(img, pattern):
    """cv2.add(u8, u8): min(a + b, 255)."""
    return np.minimum(img.astype(np.int32) + pattern.astype(np.int32), 255).astype(np.uint8)


def blob_f32(imgs, pixel_means=PIXEL_MEANS, flip=False):
    """prep_im_for_blob at scale 1.0 + im_list_to_blob: f32(f64(v) - mean), zero padded NHWC."""
    ims = []
    for im in imgs:
        if flip:
            im = im[:, ::-1, :]
        f = im.astype(np.float32, copy=True)
        f -= pixel_means
        ims.append(f)
    max_shape = np.array([im.shape for im in ims]).max(axis=0)
    blob = np.zeros((len(ims), max_shape[0], max_shape[1], 3), dtype=np.float32)
    for i, im in enumerate(ims):
        blob[i, 0:im.shape[0], 0:im.shape[1], :] = im
    return blob


# ---- the reference's own additive closures (lib/model/test.py:767-1572) --------------------------
def noise_uniform(img, u, high):
    """img_as_float(img) + np.random.uniform(0, high) given its random_sample draws u (cv2.add on
    float64: plain add)."""
    return img_as_float(img) + (0.0 + high * np.asarray(u, np.float64))


def noise_gamma(img, g, scale):
    """x + scipy gamma.rvs(1.99, loc=0, scale) given standard_gamma(1.99) draws g."""
    return img_as_float(img) + (np.asarray(g, np.float64) * scale + 0.0)


def noise_rayleigh(img, r, scale):
    """x + scipy rayleigh.rvs(loc=0, scale) given sqrt(chisquare(2)) draws r."""
    return img_as_float(img) + (np.asarray(r, np.float64) * scale + 0.0)


def brownian_walk(z, dt):
    """B = concat([0], cumsum(sqrt(dt) * z)) for the n-1 normals z (np.cumsum: sequential)."""
    dB = np.sqrt(dt) * np.asarray(z, np.float64)
    return np.concatenate((np.zeros(1), np.cumsum(dB)))


def noise_brownian(img, z, dt):
    """cv2.add(img, (B * 255).astype(np.uint8).reshape(img.shape)) (u8 + u8 saturating)."""
    pat = to_u8(brownian_walk(z, dt) * 255).reshape(img.shape)
    return add_saturate(img, pat)
