#!/opt/conda/bin/python3.9
"""Generate the golden fixtures under tests/golden/ (run in the build container only).

Interpreter: /opt/conda/bin/python3.9 with scikit-image 0.18.3, PyWavelets 1.1.1, numpy 1.26.4.
The reference pins skimage 0.14.2 / pywt 1.0.3 / numpy 1.16.6 (requirements.txt:118,151,160);
random_noise's algorithm is unchanged between 0.14.2 and 0.18.3, and the denoise_wavelet wrapper
is emulated with 0.14.2 semantics (inner and outer clip to [0, 1]) around
0.18.3's `_wavelet_threshold`.  The reference's own modules cannot be imported here (cv2 is
absent: an ordinary ModuleNotFoundError), so the fixtures come from the third-party library
the reference calls, at the reference's call signatures:

  random_noise(img, mode='gaussian', var=v)          lib/model/test.py:292 etc.
  random_noise(img, mode='s&p', amount=p)            lib/model/test.py:464 etc.
  random_noise(img, mode='speckle', var=v)           lib/model/test.py:580 etc.
  random_noise(img, mode='poisson')                  lib/model/test.py:350
  denoise_wavelet(im, method='BayesShrink', mode='soft', wavelet='bior1.5',
                  multichannel=True, convert2ycbcr=True)            lib/model/test.py:197
  denoise_wavelet(..., wavelet_levels=3) (default db1)  minibatch_before_curvelet.py:85-87
  linspace/sin periodic pattern                      lib/model/test.py:1284-1286
  uniform / gamma / rayleigh / brownian closures     lib/model/test.py:767-1572 (scipy.stats 1.7.1)
  blob: astype(f32) -= PIXEL_MEANS                   lib/utils/blob.py:35-36

Random fields are NOT stored: every case records the numpy legacy seed, and the tests re-draw the
field with np.random.RandomState (MT19937 legacy streams are stable across numpy versions).
Inputs are integer-generated (make_img) or PIL-decoded crops of the reference's data/demo JPEGs
(stored as bytes).  Outputs are stored small (u8 crops) or as SHA-256 of the full array.

  /opt/conda/bin/python3.9 tests/golden/make_fixtures.py
"""
import hashlib
import json
import sys
from pathlib import Path

import numpy as np
import pywt
import skimage
from skimage import color
from skimage.restoration._denoise import _wavelet_threshold
from skimage.util import img_as_float, random_noise

OUT = Path(__file__).resolve().parent
DEMO = Path("/root/reference/data/demo")


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def make_img(h, w, seed):
    """integer-only synthetic BGR image (no float ops: identical under any numpy)."""
    rs = np.random.RandomState(seed)
    y, x = np.mgrid[0:h, 0:w]
    base = (x * 5 + y * 3) % 200 + ((x // 16 + y // 16) % 2) * 40
    img = base[..., None] + rs.randint(-30, 31, size=(h, w, 3))
    return np.clip(img, 0, 255).astype(np.uint8)


def demo_crop(name, y0, x0, h, w):
    from PIL import Image
    rgb = np.asarray(Image.open(DEMO / name).convert("RGB"))
    return np.ascontiguousarray(rgb[y0:y0 + h, x0:x0 + w, ::-1])  # BGR like cv2.imread


def u8(x):
    return (255 * x).astype(np.uint8)


def denoise_wavelet_0142(image, wavelet="db1", wavelet_levels=None):
    """skimage 0.14.2 denoise_wavelet(image, method='BayesShrink', mode='soft', wavelet=...,
    multichannel=True, convert2ycbcr=True, wavelet_levels=...): inner clip [0, 1] per channel,
    outer clip [0, 1] after ycbcr2rgb."""
    image = img_as_float(image)
    out = color.rgb2ycbcr(image)
    for i in range(3):
        mn, mx = out[..., i].min(), out[..., i].max()
        channel = out[..., i] - mn
        channel /= mx - mn
        ch = _wavelet_threshold(channel, wavelet=wavelet, method="BayesShrink", sigma=None,
                                mode="soft", wavelet_levels=wavelet_levels)
        ch = np.clip(ch, 0, 1)
        out[..., i] = ch * (mx - mn)
        out[..., i] += mn
    out = color.ycbcr2rgb(out)
    return np.clip(out, 0, 1)


def main():
    manifest = {"generator": "tests/golden/make_fixtures.py",
                "versions": {"skimage": skimage.__version__, "pywt": pywt.__version__,
                             "numpy": np.__version__}}
    arrays = {}

    # ---------------- inputs ----------------
    imgs = {
        "syn24x40": make_img(24, 40, 11),
        "demo24x40": demo_crop("000456.jpg", 100, 120, 24, 40),
    }
    for k, v in imgs.items():
        arrays[f"in_{k}"] = v

    # ---------------- random_noise (replayable by seed) ----------------
    cases = []
    for iname, img in imgs.items():
        for mode, kw in (("gaussian", {"var": 0.1}), ("gaussian", {"var": 1.0}),
                         ("speckle", {"var": 0.5}), ("speckle", {"var": 2.0}),
                         ("s&p", {"amount": 0.4}), ("s&p", {"amount": 0.8}),
                         ("poisson", {})):
            seed = 1000 + len(cases)
            out = random_noise(img, mode=mode, seed=seed, **kw)
            key = f"noise{len(cases)}"
            arrays[key + "_u8"] = u8(out)
            cases.append({"key": key, "input": iname, "mode": mode, "kw": kw, "seed": seed,
                          "sha_f64": sha(out.astype(np.float64))})
    # full-size 600x1000 (inputs regenerated from make_img on the GPU box)
    big = make_img(600, 1000, 5)
    manifest["big_input_sha"] = sha(big)
    for mode, kw in (("gaussian", {"var": 1.0}), ("s&p", {"amount": 0.4}),
                     ("speckle", {"var": 1.0}), ("poisson", {})):
        seed = 2000 + len(cases)
        out = random_noise(big, mode=mode, seed=seed, **kw)
        cases.append({"key": None, "input": "big600x1000", "mode": mode, "kw": kw, "seed": seed,
                      "sha_u8": sha(u8(out)), "sha_f64": sha(out)})
    manifest["noise"] = cases

    # ---------------- the reference's own additive closures (scipy.stats + numpy) ----------------
    # test.py:767-903 (uniform), 1300-1437 (gamma, a = 1.99), 1439-1572 (rayleigh),
    # 905-1126 (brownian): the closure arithmetic restated line by line with the same calls.
    from scipy.stats import gamma as sp_gamma, rayleigh as sp_rayleigh
    add = []
    for iname, img in imgs.items():
        image = img_as_float(img)
        for mode, level in (("uniform", 0.2), ("uniform", 1.2), ("gamma", 0.05), ("gamma", 0.2),
                            ("rayleigh", 0.1), ("rayleigh", 0.3), ("brownian", 0.9),
                            ("brownian", 0.009)):
            seed = 3000 + len(add)
            np.random.seed(seed)
            if mode == "uniform":
                arr = image + np.random.uniform(low=0., high=level, size=img.shape)  # cv2.add
                o8 = (255 * arr).astype(np.uint8)
            elif mode == "gamma":
                arr = image + sp_gamma.rvs(1.99, loc=0., scale=level, size=image.shape)
                o8 = (arr * 255).astype(np.uint8)
            elif mode == "rayleigh":
                arr = image + sp_rayleigh.rvs(loc=0., scale=level, size=image.shape)
                o8 = (arr * 255).astype(np.uint8)
            else:
                h, w = img.shape[:2]
                n = img.size
                dB = np.sqrt(level) * np.random.normal(size=(n - 1,))
                arr = np.concatenate((np.zeros(shape=(1,)), np.cumsum(dB)))
                brownian = (arr * 255).astype(np.uint8).reshape(h, w, 3)
                o8 = np.minimum(img.astype(np.int32) + brownian, 255).astype(np.uint8)  # cv2.add
            key = f"add{len(add)}"
            arrays[key + "_u8"] = o8
            add.append({"key": key, "input": iname, "mode": mode, "level": level, "seed": seed,
                        "sha_f64": sha(np.ascontiguousarray(arr, np.float64))})
    manifest["additive"] = add

    # ---------------- periodic pattern (numpy linspace / sin / uint8 cast) ----------------
    per = []
    for (h, w), A in (((24, 40), np.pi), ((24, 40), 100.0), ((24, 40), "size"),
                      ((600, 1000), np.pi), ((600, 1000), 100.0), ((600, 1000), "size")):
        size = h * w * 3
        amp = float(size) if A == "size" else float(A)
        t = np.linspace(-amp, amp, size)
        y = np.sin(t) * 255
        pat = y.astype(np.uint8).reshape(h, w, 3)
        # elements whose 255*sin(t) lies within 1e-9 of an integer may round differently under
        # another libm; the tests mask them
        near = np.abs(y - np.round(y)) < 1e-9
        per.append({"h": h, "w": w, "amp": amp, "sha": sha(pat),
                    "near_int_idx": np.flatnonzero(near).tolist()})
        if h == 24:
            arrays[f"periodic_{len(per) - 1}"] = pat
    manifest["periodic"] = per

    # ---------------- blob LUT (astype(f32) -= PIXEL_MEANS) ----------------
    means = np.array([[[102.9801, 115.9465, 122.7717]]])
    v = np.arange(256, dtype=np.uint8).reshape(1, 256, 1).repeat(3, axis=2)
    f = v.astype(np.float32, copy=True)
    f -= means
    arrays["blob_lut"] = f[0].T.copy()  # (3, 256) float32

    # ---------------- pywt DWT restatement pins ----------------
    rs = np.random.RandomState(7)
    a = rs.rand(19, 26)
    dw = []
    for wname, lev in (("bior1.5", 2), ("db1", 3)):
        co = pywt.wavedecn(a, wname, mode="symmetric", level=lev)
        arrays[f"dwt_in"] = a
        arrays[f"dwt_{wname}_a"] = co[0]
        for li, d in enumerate(co[1:]):
            for kk, vv in d.items():
                arrays[f"dwt_{wname}_L{li}_{kk}"] = vv
        rec = pywt.waverecn(co, wname, mode="symmetric")
        arrays[f"dwt_{wname}_rec"] = rec
        dw.append({"wavelet": wname, "level": lev, "keys": sorted(co[1].keys())})
    manifest["dwt"] = dw
    manifest["dwt_max_level"] = {f"{n}_{w}": pywt.dwt_max_level(n, pywt.Wavelet(w).dec_len)
                                 for n in (24, 40, 64, 96, 120, 200, 300, 600, 1000)
                                 for w in ("bior1.5", "db1")}

    # ---------------- denoise_wavelet (0.14.2 wrapper semantics) ----------------
    wv = []
    wimgs = {
        "syn40x56": make_img(40, 56, 21),
        "demo48x64": demo_crop("001150.jpg", 60, 90, 48, 64),
        "syn64x96": make_img(64, 96, 22),
    }
    for k, v in wimgs.items():
        arrays[f"in_{k}"] = v
    for iname, img in wimgs.items():
        for wname, lev in (("bior1.5", None), ("db1", 3)):
            out = denoise_wavelet_0142(img, wavelet=wname, wavelet_levels=lev)
            key = f"wav{len(wv)}"
            arrays[key + "_f32"] = out.astype(np.float32)
            arrays[key + "_u8"] = u8(out)
            wv.append({"key": key, "input": iname, "wavelet": wname, "levels": lev})
    # wavelet on a noisy input (the reference's usual case: random_noise -> U8 -> wavelet)
    noisy = u8(random_noise(wimgs["syn64x96"], mode="gaussian", var=0.1, seed=31))
    arrays["in_noisy64x96"] = noisy
    for wname, lev in (("bior1.5", None), ("db1", 3)):
        out = denoise_wavelet_0142(noisy, wavelet=wname, wavelet_levels=lev)
        key = f"wav{len(wv)}"
        arrays[key + "_f32"] = out.astype(np.float32)
        arrays[key + "_u8"] = u8(out)
        wv.append({"key": key, "input": "noisy64x96", "wavelet": wname, "levels": lev})
    # full size: u8 sha + crops + per-channel sums
    bign = u8(random_noise(big, mode="gaussian", var=0.1, seed=41))
    manifest["big_noisy_sha"] = sha(bign)
    for wname, lev in (("bior1.5", None), ("db1", 3)):
        out = denoise_wavelet_0142(bign, wavelet=wname, wavelet_levels=lev)
        o8 = u8(out)
        key = f"wavbig_{wname}"
        arrays[key + "_crop"] = np.stack([o8[:16, :16], o8[292:308, 492:508], o8[-16:, -16:]])
        arrays[key + "_f32crop"] = np.stack([out[:16, :16], out[292:308, 492:508],
                                             out[-16:, -16:]]).astype(np.float32)
        wv.append({"key": key, "input": "big_noisy600x1000", "wavelet": wname, "levels": lev,
                   "sha_u8": sha(o8), "sum_u8": o8.reshape(-1, 3).sum(0).tolist()})
    manifest["wavelet"] = wv

    np.savez_compressed(OUT / "golden.npz", **arrays)
    (OUT / "golden.json").write_text(json.dumps(manifest, indent=1))
    tot = (OUT / "golden.npz").stat().st_size
    print(f"wrote golden.npz ({tot / 1024:.1f} KiB, {len(arrays)} arrays) and golden.json")


if __name__ == "__main__":
    sys.exit(main())
