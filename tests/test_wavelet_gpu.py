"""GPU parity of the wavelet denoiser vs the golden fixtures and the numpy oracle.

Tolerance (north star): |X' - reference| <= 1e-5 before the U8 cast; U8 outputs may differ by one
LSB only where 255*X' lies within 255e-5 of an integer (the fp32 pipeline vs fp64 reference).
"""
import json
from pathlib import Path

import numpy as np
import pytest

from test_oracle import make_img

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"
TOL = 1e-5


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD / "golden.npz", allow_pickle=False), json.loads((GOLD / "golden.json").read_text())


def run(img, wavelet, levels, f64=False):
    import torch
    import idn
    x = torch.from_numpy(np.ascontiguousarray(img)).cuda()
    if f64:
        x = x.double() / 255.0 if img.dtype == np.uint8 else x
    u8, f32 = idn.ops.denoise_wavelet(x, wavelet, levels, out="both")
    return u8.cpu().numpy(), f32.cpu().numpy().astype(np.float64)


def check_u8(u8, ref_f, ref_u8):
    d = u8.astype(int) - ref_u8.astype(int)
    assert np.abs(d).max() <= 1
    near = np.abs(255 * ref_f - np.round(255 * ref_f)) < 255 * TOL + 1e-9
    assert np.all(near[d != 0]), "U8 mismatch away from an integer boundary"


def test_wavelet_crops_vs_fixtures(dev, gold):
    g, m = gold
    for case in m["wavelet"]:
        if case["input"].startswith("big"):
            continue
        img = g["in_" + case["input"]]
        u8, f = run(img, case["wavelet"], case["levels"])
        ref = g[case["key"] + "_f32"].astype(np.float64)
        assert np.abs(f - ref).max() <= TOL, case
        check_u8(u8, ref, g[case["key"] + "_u8"])


def test_wavelet_full_size_vs_fixtures(dev, gold):
    import oracle
    g, m = gold
    big = make_img(600, 1000, 5)
    noisy = oracle.sk.to_u8(255 * oracle.sk.noise_gaussian(
        big, np.random.RandomState(41).normal(0, 0.1 ** 0.5, big.shape)))
    for case in m["wavelet"]:
        if not case["input"].startswith("big"):
            continue
        u8, f = run(noisy, case["wavelet"], case["levels"])
        crops_f = np.stack([f[:16, :16], f[292:308, 492:508], f[-16:, -16:]])
        assert np.abs(crops_f - g[case["key"] + "_f32crop"]).max() <= TOL
        ref = oracle.wavelet.denoise_wavelet(noisy, case["wavelet"], case["levels"])
        assert np.abs(f - ref).max() <= TOL
        check_u8(u8, ref, oracle.sk.to_u8(255 * ref))


def test_wavelet_f64_input_and_batch(dev):
    """the reference's f64 branches (random_noise output straight into denoise_wavelet), batched"""
    import torch
    import idn
    import oracle
    imgs = np.stack([make_img(120, 200, s) for s in (3, 4, 5)])
    f64 = np.clip(imgs / 255.0 + np.random.RandomState(0).normal(0, 0.2, imgs.shape), 0, 1)
    x = torch.from_numpy(f64).cuda()
    for wavelet, levels in (("bior1.5", None), ("db1", 3), ("db1", None)):
        u8, f = idn.ops.denoise_wavelet(x, wavelet, levels, out="both")
        f = f.cpu().numpy()
        for i in range(3):
            ref = oracle.wavelet.denoise_wavelet(f64[i], wavelet, levels)
            assert np.abs(f[i] - ref).max() <= TOL
            check_u8(u8[i].cpu().numpy(), ref, oracle.sk.to_u8(255 * ref))


@pytest.mark.parametrize("shape", [(37, 53), (9, 11), (64, 17)])
def test_wavelet_odd_shapes(dev, shape):
    import oracle
    img = make_img(*shape, 8)
    for wavelet, levels in (("bior1.5", None), ("db1", 2)):
        u8, f = run(img, wavelet, levels)
        ref = oracle.wavelet.denoise_wavelet(img, wavelet, levels)
        assert np.abs(f - ref).max() <= TOL
        check_u8(u8, ref, oracle.sk.to_u8(255 * ref))


@pytest.mark.parametrize("shape,levels", [((120, 200), 3), ((64, 96), 2), ((30, 50), 1),
                                          ((600, 1000), 3), ((48, 40), None)])
@pytest.mark.parametrize("f64", [False, True])
def test_wavelet_haar_fused_matches_general(dev, monkeypatch, shape, levels, f64):
    """the block-local Haar path (2^L-divisible sizes) agrees with the general multi-pass path:
    identical coefficients, only the sum-of-squares order differs (thresholds to a few ulps)"""
    import oracle
    img = make_img(*shape, 11)
    if f64:
        img = np.clip(img / 255.0 + np.random.RandomState(1).normal(0, 0.1, img.shape), 0, 1)
    u8a, fa = run(img, "db1", levels)
    monkeypatch.setenv("IDN_WAVELET_FUSED", "0")
    u8b, fb = run(img, "db1", levels)
    assert np.abs(fa - fb).max() <= 1e-6
    d = u8a.astype(int) - u8b.astype(int)
    assert np.abs(d).max() <= 1 and (d != 0).mean() < 1e-4
    if shape[0] * shape[1] <= 24000:
        ref = oracle.wavelet.denoise_wavelet(img, "db1", levels)
        assert np.abs(fa - ref).max() <= TOL
