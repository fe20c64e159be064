"""CPU: pin the oracle (oracle/) against the golden fixtures and independent cross-checks.

  * random_noise restatement (replayed numpy legacy fields) vs skimage 0.18.3 outputs
  * periodic pattern vs numpy linspace/sin/uint8 fixture hashes (libm near-integer cases masked)
  * blob LUT vs numpy's `astype(f32) -= PIXEL_MEANS`
  * DWT / denoise_wavelet restatement vs pywt 1.1.1 / skimage fixtures (0.14.2 wrapper semantics)
  * OpenCV filter restatement (oracle/filters.c) vs scipy.ndimage
"""
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

import oracle
from oracle import sk

GOLD = Path(__file__).resolve().parent / "golden"


@pytest.fixture(scope="module")
def gold():
    g = np.load(GOLD / "golden.npz", allow_pickle=False)
    m = json.loads((GOLD / "golden.json").read_text())
    return g, m


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def make_img(h, w, seed):
    """same integer-only generator as tests/golden/make_fixtures.py"""
    rs = np.random.RandomState(seed)
    y, x = np.mgrid[0:h, 0:w]
    base = (x * 5 + y * 3) % 200 + ((x // 16 + y // 16) % 2) * 40
    img = base[..., None] + rs.randint(-30, 31, size=(h, w, 3))
    return np.clip(img, 0, 255).astype(np.uint8)


def additive_draws(mode, seed, img):
    """numpy's unit draws of the additive closures for (mode, seed): the replay field
    (brownian: element e holds z[e-1], element 0 unused)"""
    rs = np.random.RandomState(seed)
    if mode == "uniform":
        return rs.random_sample(img.shape)
    if mode == "gamma":
        return rs.standard_gamma(1.99, img.shape)
    if mode == "rayleigh":
        return np.sqrt(rs.chisquare(2, img.shape))
    f = np.zeros(img.size)
    f[1:] = rs.normal(size=img.size - 1)
    return f.reshape(img.shape)


def additive_oracle(mode, level, img, field):
    """(u8, f64) of the oracle restatement given the replay field"""
    if mode == "uniform":
        out = sk.noise_uniform(img, field, level)
    elif mode == "gamma":
        out = sk.noise_gamma(img, field, level)
    elif mode == "rayleigh":
        out = sk.noise_rayleigh(img, field, level)
    else:
        z = field.reshape(-1)[1:]
        return sk.noise_brownian(img, z, level), sk.brownian_walk(z, level)
    return sk.to_u8(255 * out), out


def replay_field(mode, kw, seed, img):
    """re-draw the random field skimage's random_noise drew for (mode, seed)"""
    rs = np.random.RandomState(seed)
    shape = img.shape
    if mode in ("gaussian", "speckle"):
        return rs.normal(0.0, kw["var"] ** 0.5, shape)
    if mode == "s&p":
        return np.stack([rs.random_sample(shape), rs.random_sample(shape)])
    if mode == "poisson":
        return rs.poisson(sk.poisson_lambda(img)).astype(np.float64)
    raise ValueError(mode)


def oracle_noise(mode, kw, img, field):
    if mode == "gaussian":
        return sk.noise_gaussian(img, field)
    if mode == "speckle":
        return sk.noise_speckle(img, field)
    if mode == "s&p":
        return sk.noise_sap(img, field[0], field[1], kw["amount"])
    return sk.noise_poisson(img, field)


def test_big_input_generator(gold):
    _, m = gold
    assert sha(make_img(600, 1000, 5)) == m["big_input_sha"]


def test_random_noise_small(gold):
    g, m = gold
    for case in m["noise"]:
        if case["key"] is None:
            continue
        img = g["in_" + case["input"]]
        field = replay_field(case["mode"], case["kw"], case["seed"], img)
        out = oracle_noise(case["mode"], case["kw"], img, field)
        assert sha(out) == case["sha_f64"], case
        assert np.array_equal(sk.to_u8(255 * out), g[case["key"] + "_u8"]), case


def test_random_noise_full_size(gold):
    _, m = gold
    big = make_img(600, 1000, 5)
    for case in m["noise"]:
        if case["key"] is not None:
            continue
        field = replay_field(case["mode"], case["kw"], case["seed"], big)
        out = oracle_noise(case["mode"], case["kw"], big, field)
        assert sha(out) == case["sha_f64"], case
        assert sha(sk.to_u8(255 * out)) == case["sha_u8"], case


def test_to_u8_cast_semantics():
    y = np.array([0.0, 0.99, 1.0, 254.999, 255.0, 255.7, 256.0, 300.7, -1.0, -127.5, -0.5, np.nan])
    assert sk.to_u8(y).tolist() == [0, 0, 1, 254, 255, 255, 0, 44, 255, 129, 0, 0]
    # in-range values agree with numpy's own cast
    r = np.random.RandomState(0).uniform(0, 255.999, 10000)
    assert np.array_equal(sk.to_u8(r), r.astype(np.uint8))
    # img_as_float round trip loses exactly the 24 documented values
    v = np.arange(256, dtype=np.uint8)
    lost = np.flatnonzero(sk.to_u8(255 * sk.img_as_float(v)) != v)
    assert lost.tolist() == [33, 37, 41, 45, 49, 53, 57, 61, 66, 74, 82, 90, 98, 106, 114, 122,
                             132, 148, 164, 180, 196, 212, 228, 244]


def test_periodic_pattern(gold):
    g, m = gold
    for i, case in enumerate(m["periodic"]):
        pat = sk.periodic_pattern(case["h"], case["w"], 3, case["amp"])
        if sha(pat) != case["sha"]:
            # another libm may round sin() differently only where 255*sin(t) is ~integer
            key = f"periodic_{i}"
            assert key in g, "full-size pattern mismatch outside near-integer elements"
        if f"periodic_{i}" in g:
            ref = g[f"periodic_{i}"].reshape(-1)
            got = pat.reshape(-1)
            diff = np.flatnonzero(got != ref)
            assert set(diff.tolist()) <= set(case["near_int_idx"])


def test_blob_lut(gold):
    g, _ = gold
    v = np.arange(256, dtype=np.uint8).reshape(1, 256, 1).repeat(3, axis=2)
    blob = sk.blob_f32([v])
    assert np.array_equal(blob[0, 0].T, g["blob_lut"])
    # the naive f32 arithmetic differs (why the kernel subtracts in f64)
    naive = v.astype(np.float32) - sk.PIXEL_MEANS.astype(np.float32)
    assert (naive[0].T != g["blob_lut"]).sum() > 300


def test_blob_padding_and_flip():
    a = np.random.RandomState(1).randint(0, 256, (4, 5, 3)).astype(np.uint8)
    b = np.random.RandomState(2).randint(0, 256, (6, 3, 3)).astype(np.uint8)
    blob = sk.blob_f32([a, b])
    assert blob.shape == (2, 6, 5, 3)
    assert np.all(blob[0, 4:] == 0) and np.all(blob[1, :, 3:] == 0)
    fl = sk.blob_f32([a], flip=True)
    assert np.array_equal(fl[0], sk.blob_f32([a[:, ::-1]])[0])


def test_dwt_restatement(gold):
    g, m = gold
    a = g["dwt_in"]
    for case in m["dwt"]:
        w, lev = case["wavelet"], case["level"]
        co = oracle.wavelet.wavedecn(a, w, lev)
        np.testing.assert_allclose(co[0], g[f"dwt_{w}_a"], rtol=0, atol=1e-13)
        for li in range(lev):
            for k in case["keys"]:
                np.testing.assert_allclose(co[1 + li][k], g[f"dwt_{w}_L{li}_{k}"], rtol=0, atol=1e-13)
        rec = oracle.wavelet.waverecn(co, w)
        np.testing.assert_allclose(rec, g[f"dwt_{w}_rec"], rtol=0, atol=1e-13)
    for key, lvl in m["dwt_max_level"].items():
        n, w = key.split("_")
        assert oracle.wavelet.dwt_max_level(int(n), len(oracle.wavelet.FILTERS[w][0])) == lvl


@pytest.mark.parametrize("shape", [(37, 53), (8, 9), (600, 1000)])
def test_bior15_finest_dd_is_a_2x2_combination(shape):
    """bior1.5's analysis highpass has two taps, so each level-1 dd coefficient (pywt dwtn: axis 0,
    then axis 1) is the 2x2 combination of the samples at rows 2i-4, 2i-3 and columns 2j-4, 2j-3
    ('symmetric' indices) in the op order (-S * odd) + (S * even): bit for bit.  The HIP sigma median
    recomputes its candidates this way (csrc/wavelet.hip bior_dd2x2) instead of storing the fp64
    band."""
    from oracle.wavelet import _S, _sym_index, dwtn
    x = np.random.RandomState(sum(shape)).rand(*shape)
    dd = dwtn(x, "bior1.5")["dd"]
    i = np.arange(dd.shape[0])[:, None]
    j = np.arange(dd.shape[1])[None, :]
    r0, r1 = _sym_index(2 * i - 4, shape[0]), _sym_index(2 * i - 3, shape[0])
    c0, c1 = _sym_index(2 * j - 4, shape[1]), _sym_index(2 * j - 3, shape[1])
    h0 = (-_S) * x[r1, c0] + _S * x[r0, c0]  # column highpass of both columns
    h1 = (-_S) * x[r1, c1] + _S * x[r0, c1]
    np.testing.assert_array_equal(((-_S) * h1 + _S * h0).view(np.uint64), dd.view(np.uint64))


def test_denoise_wavelet_crops(gold):
    g, m = gold
    for case in m["wavelet"]:
        if case["input"].startswith("big"):
            continue
        img = g["in_" + case["input"]]
        out = oracle.wavelet.denoise_wavelet(img, case["wavelet"], case["levels"])
        np.testing.assert_allclose(out, g[case["key"] + "_f32"], rtol=0, atol=1e-6)
        assert np.array_equal(sk.to_u8(255 * out), g[case["key"] + "_u8"])


def test_denoise_wavelet_full_size(gold):
    g, m = gold
    big = make_img(600, 1000, 5)
    noisy = sk.to_u8(255 * sk.noise_gaussian(big, np.random.RandomState(41).normal(0, 0.1 ** 0.5, big.shape)))
    assert sha(noisy) == m["big_noisy_sha"]
    for case in m["wavelet"]:
        if not case["input"].startswith("big"):
            continue
        out = oracle.wavelet.denoise_wavelet(noisy, case["wavelet"], case["levels"])
        o8 = sk.to_u8(255 * out)
        crops = np.stack([o8[:16, :16], o8[292:308, 492:508], o8[-16:, -16:]])
        f32c = np.stack([out[:16, :16], out[292:308, 492:508], out[-16:, -16:]])
        np.testing.assert_allclose(f32c, g[case["key"] + "_f32crop"], rtol=0, atol=1e-6)
        assert np.array_equal(crops, g[case["key"] + "_crop"])
        assert sha(o8) == case["sha_u8"]


@pytest.mark.parametrize("k", [3, 5])
def test_cv_filters_vs_scipy(k):
    import scipy.ndimage as nd
    img = np.random.RandomState(k).randint(0, 256, (2, 29, 41, 3)).astype(np.uint8)
    a = np.array([1, 2, 1]) if k == 3 else np.array([1, 4, 6, 4, 1])
    w2 = np.outer(a, a)
    sh = 4 if k == 3 else 8
    for i in range(2):
        S = np.stack([nd.correlate(img[i, ..., c].astype(np.int64), w2, mode="mirror") for c in range(3)], -1)
        assert np.array_equal(((S + (1 << (sh - 1))) >> sh).astype(np.uint8),
                              oracle.cv.gaussian_blur(img, k)[i])
        ref = nd.median_filter(img[i], size=(k, k, 1), mode="nearest")
        assert np.array_equal(ref, oracle.cv.median_blur(img, k)[i])
        if k == 3:
            S = np.stack([nd.correlate(img[i, ..., c].astype(np.int64), np.ones((3, 3), np.int64),
                                       mode="mirror") for c in range(3)], -1)
            assert np.array_equal(((2 * S + 9) // 18).astype(np.uint8), oracle.cv.blur(img, 3)[i])


def test_cv_filters_tiny_images():
    """h or w smaller than the kernel: REFLECT_101 repeats, REPLICATE clamps"""
    import scipy.ndimage as nd
    for h, w in ((1, 7), (2, 2), (3, 1), (2, 9)):
        img = np.random.RandomState(h * 10 + w).randint(0, 256, (h, w, 3)).astype(np.uint8)
        ref = nd.median_filter(img, size=(5, 5, 1), mode="nearest")
        assert np.array_equal(ref, oracle.cv.median_blur(img, 5))
        a = np.array([1, 4, 6, 4, 1])
        S = np.stack([nd.correlate(img[..., c].astype(np.int64), np.outer(a, a), mode="mirror")
                      for c in range(3)], -1)
        if h > 2 and w > 2:  # scipy 'mirror' and OpenCV REFLECT_101 agree when len >= 3
            assert np.array_equal(((S + 128) >> 8).astype(np.uint8), oracle.cv.gaussian_blur(img, 5))


def test_bilateral_oracle_self_consistent():
    img = np.random.RandomState(3).randint(0, 256, (23, 31, 3)).astype(np.uint8)
    for sc, ss in ((20, 100), (75, 75)):
        b = oracle.cv.bilateral_filter(img, 9, sc, ss)
        f = oracle.cv.bilateral_prefilter_f32(img, 9, sc, ss)
        assert np.abs(b.astype(np.float64) - f).max() <= 0.5 + 1e-3


def test_cvf_float64_filters_vs_scipy():
    """oracle/cvf.py float64 Gaussian/box (cv2 summation order) vs scipy.ndimage (mirror)."""
    import numpy as np
    import scipy.ndimage as nd
    import oracle
    x = np.random.RandomState(5).rand(2, 23, 31, 3)
    for k, w in ((3, np.array([1, 2, 1]) / 4.0), (5, np.array([1, 4, 6, 4, 1]) / 16.0)):
        ref = nd.correlate1d(nd.correlate1d(x, w, axis=2, mode="mirror"), w, axis=1, mode="mirror")
        assert np.abs(oracle.cvf.gaussian_blur_f64(x, k) - ref).max() < 1e-15
    ref = nd.uniform_filter(x, size=(1, 3, 3, 1), mode="mirror")
    assert np.abs(oracle.cvf.blur_f64(x, 3) - ref).max() < 1e-14
    one = x[:, :1, :1]
    assert np.allclose(oracle.cvf.blur_f64(one, 3), one)


def test_cvf_resize_vs_torch_bilinear():
    """INTER_LINEAR restatement vs torch bilinear (align_corners=False, same sampling grid) on
    upscales, where both clamp identically (OpenCV rounds the source coordinate to float32 before
    flooring, torch keeps its own float formula: agreement to ~1e-5 relative)."""
    import numpy as np
    import torch
    import oracle
    rs = np.random.RandomState(6)
    for s, hw in ((1.6, (40, 55)), (2.0, (37, 53)), (1.25, (40, 56))):
        x = rs.uniform(-128, 128, size=(*hw, 3)).astype(np.float32)
        r = oracle.cvf.resize_linear_f32(x, s, s)
        t = torch.nn.functional.interpolate(torch.from_numpy(x).permute(2, 0, 1)[None],
                                            scale_factor=s, mode="bilinear", align_corners=False,
                                            recompute_scale_factor=False)[0].permute(1, 2, 0).numpy()
        assert r.shape == t.shape
        assert np.abs(r - t).max() < 4e-3  # |x| <= 128: coefficient rounding differs at ~1e-5 rel
    assert np.array_equal(oracle.cvf.resize_linear_f32(x, 1.0, 1.0), x)


def test_bloom_circle_tables_agree():
    """Two restatements of cv2.circle(LINE_8, filled): the oracle's span drawing and the span
    table the GPU kernel consumes (idn.automold.circle_half_widths)."""
    import numpy as np
    import oracle
    from idn import automold
    for R in (0, 1, 2, 3, 7, 8, 27, 64, 125, 399):
        n = 2 * R + 3
        img = np.zeros((n, n, 1), np.uint8)
        oracle.automold.circle_fill(img, (R + 1, R + 1), R, (1,))
        half = automold.circle_half_widths(R)
        for t in range(-R - 1, R + 2):
            row = img[R + 1 + t, :, 0]
            hw = half[abs(t)] if abs(t) <= R else -1
            expect = np.zeros(n, np.uint8)
            if hw >= 0:
                expect[R + 1 - hw: R + 2 + hw] = 1
            assert np.array_equal(row, expect), (R, t)


def test_additive_noises_vs_fixtures(gold):
    """uniform / gamma / rayleigh / brownian closures (test.py:767-1572) restated in oracle/sk.py,
    pinned to fixtures computed with scipy.stats 1.7.1 + numpy at the reference's calls"""
    g, m = gold
    assert len(m["additive"]) == 16
    for case in m["additive"]:
        img = g["in_" + case["input"]]
        field = additive_draws(case["mode"], case["seed"], img)
        u8, f = additive_oracle(case["mode"], case["level"], img, field)
        assert np.array_equal(u8, g[case["key"] + "_u8"]), case
        assert sha(np.ascontiguousarray(f, np.float64)) == case["sha_f64"], case


def test_fast_cpu_baseline_bitexact_with_scalar_oracle():
    """bench.py's cpu_baseline times oracle/baseline_fast.c; it must compute the same filter."""
    rs = np.random.RandomState(4)
    for shape in [(2, 120, 200, 3), (1, 5, 6, 3), (1, 33, 17, 3), (2, 9, 40, 1)]:
        img = rs.randint(0, 256, size=shape).astype(np.uint8)
        for k in (3, 5):
            assert np.array_equal(oracle.cv.gaussian_blur_fast(img, k),
                                  oracle.cv.gaussian_blur(img, k)), (shape, k)


def test_key_ties_fixture_is_reproduced():
    """tests/golden/make_key_ties.py (the search over all 2^24 RGB triples for exact YCbCr ties
    whose fp64 values differ, at each channel's extremes) reproduces the triples the GPU test
    test_wavelet_color_minmax_key_ties places"""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "make_key_ties", Path(__file__).parent / "golden" / "make_key_ties.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    from test_wavelet_gpu import _KEY_TIES
    assert mod.find_ties() == _KEY_TIES
