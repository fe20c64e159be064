"""GPU parity of the wavelet denoiser vs the golden fixtures and the numpy oracle.

Tolerance (north star): |X' - reference| <= 1e-5 before the U8 cast; U8 outputs may differ by one
LSB only where 255*X' lies within 255e-5 of an integer (our fp64 summation order and the exact
quotients differ from numpy's in the last bits; the cast is discontinuous at integers).
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


def _stats_after(x, levels):
    """denoise_wavelet(db1) on device batch x; returns (u8, f32, per-image stats blocks)"""
    import torch
    import idn
    from idn import _lib, ops
    u8, f = ops.denoise_wavelet(x, "db1", levels, out="both")
    n, h, w, _ = x.shape
    off = _lib.load().idn_wavelet_stats_offset(n, h, w, ops.WAVELETS["db1"], levels)
    ws = ops._WS_CACHE[(str(x.device), torch.cuda.current_stream(x.device).cuda_stream)]
    st = ws[off:off + n * 256 * 8].view(torch.float64).view(n, 256).cpu().numpy().copy()
    return u8.cpu().numpy(), f.cpu().numpy(), st


def _stat_images(h, w):
    import oracle
    rs = np.random.RandomState(7)
    yy, xx = np.mgrid[0:h, 0:w]
    ramp = ((xx * 3 + yy * 5) % 256).astype(np.uint8)
    gray = np.repeat(ramp[..., None], 3, axis=2)  # R = G = B: dd on exact bin edges, T = 0 residues
    flat = np.repeat(((xx // 16 + yy // 16) % 3 * 60).astype(np.uint8)[..., None], 3, axis=2)
    flat[..., 1] = 255 - flat[..., 1]  # piecewise constant: mostly exact zeros
    tex = make_img(h, w, 13)
    noisy = oracle.sk.to_u8(255 * oracle.sk.noise_gaussian(
        tex, rs.normal(0, 0.1 ** 0.5, tex.shape)))
    uni = rs.randint(0, 256, (h, w, 3)).astype(np.uint8)
    step = np.zeros((h, w, 3), np.uint8)
    step[:, w // 2:] = (3, 1, 2)  # |T| < 3 combinations at one column (Cb: gcd 1)
    step[h // 3:, :, 1] += 1
    # channels in {0, 255}: Y's dd of equal-channel combinations are exactly 0.5 or 1.0 (bin edges)
    binc = (rs.randint(0, 2, (h, w, 3)) * 255).astype(np.uint8)
    return np.stack([gray, flat, tex, noisy, uni, step, binc])


@pytest.mark.parametrize("levels", [3, 2])
def test_wavelet_haar_integer_stats_match_fp64(dev, monkeypatch, levels):
    """the integer statistics against wl_haar_analyze (the fp64 planes): L = 2 (wl_haar_stats,
    dd codes with exact fallback) sigma medians bit-identical; L = 3 (round 6, wl_h3_stats /
    wl_h3_sigma: sigma from the exact integer |T| of the median rank) within the analytic bound
    2.1e-12 / range of the reference's fp64 value; nonzero counts exact, sums of squares to 1e-12
    relative, outputs to rounding"""
    import torch
    x = torch.from_numpy(_stat_images(96, 160)).cuda()
    from idn import _lib
    u8a, fa, sa = _stats_after(x, levels)  # product library: integer statistics
    monkeypatch.setenv("IDN_WAVELET_INTSTATS", "0")
    monkeypatch.setenv("IDN_WAVELET_H3", "0")
    with _lib.variant("tuning"):
        u8b, fb, sb = _stats_after(x, levels)
    L = levels
    med = slice(8 + 9 * L, 8 + 9 * L + 3)
    if L == 2:
        np.testing.assert_array_equal(sa[:, med].view(np.uint64), sb[:, med].view(np.uint64))
    else:
        rng = _key_to_f64(sb[:, 203:206].view(np.uint64)) - _key_to_f64(sb[:, 200:203].view(np.uint64))
        ok = np.abs(sa[:, med] - sb[:, med]) <= 2.1e-12 / np.maximum(rng, 1e-300)
        assert np.all(ok | (np.isnan(sa[:, med]) & np.isnan(sb[:, med]))), (sa[:, med], sb[:, med])
    np.testing.assert_array_equal(sa[:, 248:251], sb[:, 248:251])
    np.testing.assert_array_equal(sa[:, 200:206].view(np.uint64), sb[:, 200:206].view(np.uint64))
    # channels whose YCbCr range is rounding noise (Cb / Cr of the gray image) are exempt: their
    # fp64-plane sums are noise, and such a channel's output is min + v * range whatever they are
    imgs = x.cpu().numpy().astype(np.float64) / 255.0
    m = np.array([[65.481, 128.553, 24.966], [-37.797, -74.203, 112.0], [112.0, -93.786, -18.214]])
    ycc = imgs @ m.T
    live = (ycc.max(axis=(1, 2)) - ycc.min(axis=(1, 2))) > 1e-6  # (n, 3)
    sq_a = sa[:, 8:8 + 9 * L].reshape(-1, 3, 3 * L)
    sq_b = sb[:, 8:8 + 9 * L].reshape(-1, 3, 3 * L)
    ok = np.abs(sq_a - sq_b) <= 1e-12 * np.abs(sq_b) + 1e-300
    assert np.all(ok[live]), np.abs(sq_a - sq_b)[live].max()
    assert np.abs(fa - fb).max() <= 1e-6
    d = u8a.astype(int) - u8b.astype(int)
    assert np.abs(d).max() <= 1 and (d != 0).mean() < 1e-4


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
    from idn import _lib
    monkeypatch.setenv("IDN_WAVELET_FUSED", "0")
    with _lib.variant("tuning"):
        u8b, fb = run(img, "db1", levels)
    assert np.abs(fa - fb).max() <= 1e-6
    d = u8a.astype(int) - u8b.astype(int)
    assert np.abs(d).max() <= 1 and (d != 0).mean() < 1e-4
    if shape[0] * shape[1] <= 24000:
        ref = oracle.wavelet.denoise_wavelet(img, "db1", levels)
        assert np.abs(fa - ref).max() <= TOL


@pytest.mark.parametrize("shape,wavelet,levels", [((600, 1000), "bior1.5", None),
                                                  ((37, 53), "bior1.5", None),
                                                  ((90, 70), "db1", 3)])
def test_wavelet_fp32_details_vs_fp64(dev, monkeypatch, shape, wavelet, levels):
    """IDN_WAVELET_FDET: ad / da bands through HBM as fp32 (default) against the all-fp64 form
    (IDN_WAVELET_FDET=0), both with the fp64 synthesis (IDN_WAVELET_S32=0) so that only the band
    storage differs; both within TOL of the oracle, and within 1e-6 of each other"""
    import oracle
    img = make_img(*shape, 17)
    from idn import _lib
    monkeypatch.setenv("IDN_WAVELET_S32", "0")
    with _lib.variant("tuning"):
        u8a, fa = run(img, wavelet, levels)
    monkeypatch.setenv("IDN_WAVELET_FDET", "0")
    with _lib.variant("tuning"):
        u8b, fb = run(img, wavelet, levels)
    assert np.abs(fa - fb).max() <= 1e-6
    d = u8a.astype(int) - u8b.astype(int)
    assert np.abs(d).max() <= 1 and (d != 0).mean() < 1e-4
    ref = oracle.wavelet.denoise_wavelet(img, wavelet, levels)
    assert np.abs(fb - ref).max() <= TOL
    check_u8(u8b, ref, oracle.sk.to_u8(255 * ref))


def _run_env(monkeypatch, img, env):
    from idn import _lib
    with monkeypatch.context() as mp:
        for k, v in env.items():
            mp.setenv(k, v)
        with _lib.variant("tuning"):
            return run(img, "bior1.5", None)


@pytest.mark.parametrize("shape", [(600, 1000), (37, 53), (9, 11), (130, 77)])
@pytest.mark.parametrize("form", ["0", "1", "2"])
def test_wavelet_bior15_synthesis_forms(dev, monkeypatch, shape, form):
    """IDN_WAVELET_SSTREAM in fp64 (IDN_WAVELET_S32=0; bit 0 level 1, bit 1 deeper levels:
    streaming wl_synth_stream vs tiled wl_synth / wl_synth_final): every mix within 1e-9 of the
    all-streaming fp64 form (the same pair arithmetic, staged differently) and within TOL of the
    oracle"""
    import oracle
    img = make_img(*shape, 29)
    u8a, fa = _run_env(monkeypatch, img, {"IDN_WAVELET_S32": "0", "IDN_WAVELET_SSTREAM": "3"})
    u8b, fb = _run_env(monkeypatch, img, {"IDN_WAVELET_S32": "0", "IDN_WAVELET_SSTREAM": form})
    assert np.abs(fa - fb).max() <= 1e-9
    d = u8a.astype(int) - u8b.astype(int)
    assert np.abs(d).max() <= 1 and (d != 0).mean() < 1e-4
    if shape[0] * shape[1] <= 24000:
        ref = oracle.wavelet.denoise_wavelet(img, "bior1.5", None)
        assert np.abs(fb - ref).max() <= TOL
        check_u8(u8b, ref, oracle.sk.to_u8(255 * ref))


@pytest.mark.parametrize("shape", [(600, 1000), (37, 53), (9, 11), (130, 77)])
@pytest.mark.parametrize("env", [{"IDN_WAVELET_S32": "0"},
                                 {"IDN_WAVELET_S32": "1", "IDN_WAVELET_SSTREAM": "2"},
                                 {"IDN_WAVELET_S32": "1", "IDN_WAVELET_SSTREAM": "1"}],
                         ids=["fp64", "f32-deeper", "f32-level1"])
def test_wavelet_bior15_fp32_synthesis(dev, monkeypatch, shape, env):
    """the product's fp32 streaming synthesis (IDN_WAVELET_S32 default on: taps, soft threshold,
    de-normalisation and YCbCr -> RGB in fp32, levels >= 2 handing fp32 reconstructions down)
    against the fp64 synthesis and against mixes with the tiled fp64 forms: within 2e-6 on the
    [0, 1] scale, U8 one LSB only at integer boundaries; the product within TOL of the oracle"""
    import oracle
    img = make_img(*shape, 31)
    u8a, fa = run(img, "bior1.5", None)
    u8b, fb = _run_env(monkeypatch, img, env)
    assert np.abs(fa - fb).max() <= 2e-6
    check_u8(u8a, fb, u8b)
    if shape[0] * shape[1] <= 24000:
        ref = oracle.wavelet.denoise_wavelet(img, "bior1.5", None)
        assert np.abs(fa - ref).max() <= TOL
        check_u8(u8a, ref, oracle.sk.to_u8(255 * ref))


@pytest.mark.parametrize("shape", [(600, 1000), (601, 999), (130, 77), (37, 53), (9, 11), (40, 1100)])
def test_wavelet_bior15_final3_bitwise(dev, monkeypatch, shape):
    """wl_synth_final3 (level 1, all three channels per thread; product) against the per-channel
    streaming kernel (IDN_WAVELET_S3=0): the same fp32 operations per output, so bit-identical U8
    and float outputs (odd sizes, several strips, L = 1 with an fp64 coarsest aa)"""
    img = make_img(*shape, 41)
    u8a, fa = run(img, "bior1.5", None)
    u8c, fc = run(img, "bior1.5", None)
    np.testing.assert_array_equal(u8a, u8c)  # deterministic
    np.testing.assert_array_equal(fa, fc)
    u8b, fb = _run_env(monkeypatch, img, {"IDN_WAVELET_S3": "0"})
    nd = int((fa != fb).sum())
    print(f"final3 vs stream: {nd} float outputs differ, max {np.abs(fa - fb).max():.3g}")
    np.testing.assert_array_equal(u8a, u8b)
    np.testing.assert_array_equal(fa, fb)


@pytest.mark.parametrize("shape", [(600, 1000), (1201, 2003), (130, 77), (40, 1100)])
def test_wavelet_bior15_final3_deeper_bitwise(dev, monkeypatch, shape):
    """wl_synth_final3<FM, false> at the deeper levels (IDN_WAVELET_S3D = 0: every level >= 2;
    product) against wl_synth_stream<false, float> (a width floor above every level): the same
    fp32 operations per reconstructed sample, so bit-identical outputs (one and several strips,
    odd sizes)"""
    img = make_img(*shape, 43)
    u8a, fa = _run_env(monkeypatch, img, {"IDN_WAVELET_S3D": "0"})
    u8b, fb = _run_env(monkeypatch, img, {"IDN_WAVELET_S3D": str(1 << 30)})
    print(f"final3 deeper vs stream: {int((fa != fb).sum())} float outputs differ")
    np.testing.assert_array_equal(u8a, u8b)
    np.testing.assert_array_equal(fa, fb)


def _bior_stats(monkeypatch, img, env):
    """bior1.5 through the tuning build under env: (u8, f32, stats block of the image)"""
    import torch
    from idn import _lib, ops
    x = torch.from_numpy(np.ascontiguousarray(img[None])).cuda()
    with monkeypatch.context() as mp:
        for k, v in env.items():
            mp.setenv(k, v)
        with _lib.variant("tuning"):
            u8, f = ops.denoise_wavelet(x, "bior1.5", None, out="both")
            off = _lib.load().idn_wavelet_stats_offset(1, img.shape[0], img.shape[1],
                                                       ops.WAVELETS["bior1.5"], -1)
    ws = ops._WS_CACHE[(str(x.device), torch.cuda.current_stream(x.device).cuda_stream)]
    st = ws[off:off + 256 * 8].view(torch.float64).cpu().numpy().copy()
    return u8[0].cpu().numpy(), f[0].cpu().numpy().astype(np.float64), st


@pytest.mark.parametrize("shape", [(600, 1000), (130, 77), (37, 53), (9, 11)])
@pytest.mark.parametrize("a32", ["1", "2", "3", "7"])
def test_wavelet_bior15_fp32_analysis(dev, monkeypatch, shape, a32):
    """IDN_WAVELET_A32 (bit 0: level 1's lowpass path aa / ad / da in fp32, the normalisation,
    column highpass and dd in fp64; bit 1: deeper levels in fp32; bit 2 (round 6, A/B form):
    level 1's normalisation and highpass in fp32 too, the finest dd's codes from the exact
    integer keys) against the fp64 analysis:
    the finest dd -- hence the sigma medians and the nonzero counts -- bit-identical, outputs
    within 2e-6, small images within TOL of the oracle"""
    import oracle
    img = make_img(*shape, 37)
    q = min(shape) // 9  # default levels (wl_layout): max(dwt_max_level - 3, 1)
    lv = max((q.bit_length() - 1 if q >= 1 else 0) - 3, 1)
    u8a, fa, sa = _bior_stats(monkeypatch, img, {"IDN_WAVELET_A32": "0"})
    u8b, fb, sb = _bior_stats(monkeypatch, img, {"IDN_WAVELET_A32": a32})
    med = slice(8 + 9 * lv, 8 + 9 * lv + 3)
    np.testing.assert_array_equal(sa[med].view(np.uint64), sb[med].view(np.uint64))
    np.testing.assert_array_equal(sa[248:251], sb[248:251])
    assert np.abs(fa - fb).max() <= 2e-6
    check_u8(u8b, fa, u8a)
    if shape[0] * shape[1] <= 24000:
        ref = oracle.wavelet.denoise_wavelet(img, "bior1.5", None)
        assert np.abs(fb - ref).max() <= TOL
        check_u8(u8b, ref, oracle.sk.to_u8(255 * ref))


def test_wavelet_bior15_n32_stat_images(dev, monkeypatch):
    """the fp32 level-1 analysis with integer-key codes (IDN_WAVELET_A32=7) against the product's
    fp64-highpass form (3) on images with exact zeros, rounding residues (gray: T = 0), |T| < 3
    combinations, bin-edge values and saturated channels -- every code the analysis cannot certify
    is set by the median workgroup from the exact fp64 key: sigma medians and nonzero counts
    bit-identical, outputs within 2e-6"""
    import torch
    from idn import _lib
    x = torch.from_numpy(np.concatenate([_stat_images(96, 160),
                                         np.stack([_clipped(96, 160, 5)])])).cuda()
    out = {}
    for a32 in ("3", "7"):
        monkeypatch.setenv("IDN_WAVELET_A32", a32)
        with _lib.variant("tuning"):
            out[a32] = _stats_after_w(x, "bior1.5", None)
    (u8a, fa, sa), (u8b, fb, sb) = out["3"], out["7"]
    lv = 1  # 96 x 160: max(dwt_max_level - 3, 1)
    med = slice(8 + 9 * lv, 8 + 9 * lv + 3)
    np.testing.assert_array_equal(sa[:, med].view(np.uint64), sb[:, med].view(np.uint64))
    np.testing.assert_array_equal(sa[:, 248:251], sb[:, 248:251])
    assert np.abs(fa - fb).max() <= 2e-6
    # U8 flips only on rounding boundaries (the flat / gray images sit on exact k / 255 values)
    check_u8(u8b, fa.astype(np.float64), u8a)


@pytest.mark.parametrize("shape", [(600, 1000), (130, 77), (37, 53)])
@pytest.mark.parametrize("src", ["u8", "f64"])
def test_wavelet_dd32_sigma_bitwise(dev, monkeypatch, shape, src):
    """IDN_WAVELET_DD32 (product 1): the level-1 dd band stored as fp32, the sigma median
    recomputing its candidates' exact |dd| from the input (bior_dd2x2 / wl_bior_dd1_key64) in
    wl_dwt_stream's fp64 op order -- against DD32=0 (the fp64 dd band the median reads back):
    sigma medians and nonzero counts bit-identical for u8 and float64 input, outputs within 2e-6"""
    import torch
    from idn import _lib, ops
    img = make_img(*shape, 41)
    x = torch.from_numpy(np.ascontiguousarray(img[None])).cuda()
    if src == "f64":
        x = x.double() * (1.0 / 255.0)
    q = min(shape) // 9
    lv = max((q.bit_length() - 1 if q >= 1 else 0) - 3, 1)
    res = {}
    for dd32 in ("0", "1"):
        with monkeypatch.context() as mp:
            mp.setenv("IDN_WAVELET_DD32", dd32)
            with _lib.variant("tuning"):
                u8, f = ops.denoise_wavelet(x, "bior1.5", None, out="both")
                off = _lib.load().idn_wavelet_stats_offset(1, shape[0], shape[1],
                                                           ops.WAVELETS["bior1.5"], -1)
        ws = ops._WS_CACHE[(str(x.device), torch.cuda.current_stream(x.device).cuda_stream)]
        st = ws[off:off + 256 * 8].view(torch.float64).cpu().numpy().copy()
        res[dd32] = (u8[0].cpu().numpy(), f[0].cpu().numpy().astype(np.float64), st)
    (u8a, fa, sa), (u8b, fb, sb) = res["0"], res["1"]
    med = slice(8 + 9 * lv, 8 + 9 * lv + 3)
    np.testing.assert_array_equal(sa[med].view(np.uint64), sb[med].view(np.uint64))
    np.testing.assert_array_equal(sa[248:251], sb[248:251])
    assert np.abs(fa - fb).max() <= 2e-6
    check_u8(u8b, fa, u8a)


@pytest.mark.parametrize("shape", [(601, 999), (37, 53), (9, 11)])
def test_wavelet_coop_normalisation_bitwise(dev, monkeypatch, shape):
    """IDN_WAVELET_COOP (the tiled analysis wl_dwt_rb, which the general Haar path uses: sizes not
    divisible by 2^L): each staged pixel normalised once (default) against the per-channel form
    (=0): the same fp64 operations per sample, so bit-identical outputs"""
    img = make_img(*shape, 23)
    u8a, fa = run(img, "db1", None)
    from idn import _lib
    monkeypatch.setenv("IDN_WAVELET_COOP", "0")
    with _lib.variant("tuning"):
        u8b, fb = run(img, "db1", None)
    np.testing.assert_array_equal(u8a, u8b)
    np.testing.assert_array_equal(fa, fb)


def _key_to_f64(k):
    k = k.astype(np.uint64)
    neg = (k >> np.uint64(63)) == 0
    bits = np.where(neg, ~k, k & np.uint64(0x7FFFFFFFFFFFFFFF))
    return bits.view(np.float64)


def test_wavelet_color_minmax_exact(dev):
    """wl_color_minmax: the per-channel YCbCr min / max in the stats block equal numpy's fp64
    rgb2ycbcr min / max bit for bit, on images whose triples tie in exact value but not in fp64
    (gray ramps: Cb / Cr), binary channels, saturated noise and uniform noise"""
    import torch
    import oracle
    from oracle.cv import matmul3_fma
    imgs = _stat_images(96, 160)
    rs = np.random.RandomState(5)
    sat = np.clip(rs.normal(128, 200, imgs.shape[1:]), 0, 255).astype(np.uint8)  # many 0 / 255
    imgs = np.concatenate([imgs, sat[None]])
    _, _, st = _stats_after(torch.from_numpy(imgs).cuda(), 2)
    for i, img in enumerate(imgs):
        ycc = matmul3_fma(img.astype(np.float64) * (1.0 / 255.0), oracle.wavelet.YCBCR_FROM_RGB,
                          post=oracle.wavelet.YCBCR_OFFSET)
        mn = _key_to_f64(st[i, 200:203].view(np.uint64))
        mx = _key_to_f64(st[i, 203:206].view(np.uint64))
        np.testing.assert_array_equal(mn.view(np.uint64), ycc.min(axis=(0, 1)).view(np.uint64))
        np.testing.assert_array_equal(mx.view(np.uint64), ycc.max(axis=(0, 1)).view(np.uint64))


# per channel (Y, Cb, Cr) and extreme (lowest, highest): two triples whose exact YCbCr values tie
# (equal integer keys 1000 M . rgb) while their fp64 values differ in the last bits -- the search
# over all 2^24 triples is tests/golden/make_key_ties.py (test_oracle.py checks it reproduces this)
_KEY_TIES = [((12, 1, 2), (1, 0, 36)), ((244, 254, 254), (255, 255, 220)),
             ((252, 255, 1), (251, 254, 0)), ((2, 4, 255), (0, 2, 253)),
             ((0, 254, 252), (1, 255, 253)), ((254, 0, 3), (255, 1, 4))]


@pytest.mark.parametrize("swap", [False, True])
def test_wavelet_color_minmax_key_ties(dev, swap):
    """wl_color_minmax evaluates the fp64 YCbCr chain on every pixel and reduces min / max per
    channel (an exact-integer-key ranking was measured slower and not shipped).  Each
    channel's min and max here is reached by two triples whose exact values tie and whose fp64
    values differ, adjacent in one thread's pixel group (either order) and again in other
    threads: the stats must equal numpy's fp64 min / max bit for bit, i.e. the kernel's chain must
    round exactly as numpy's (a chain that rounds differently picks the other triple's value)"""
    import torch
    import oracle
    from oracle.cv import matmul3_fma
    rs = np.random.RandomState(11)
    img = rs.randint(40, 201, (96, 160, 3)).astype(np.uint8)  # no pixel reaches the tied extremes
    flat = img.reshape(-1, 3)
    for j, (a, b) in enumerate(_KEY_TIES):
        pair = (b, a) if swap else (a, b)
        base = 4 * (37 * j + 5)  # one 4-pixel group: one thread, consecutive pixels
        flat[base], flat[base + 1] = pair
        flat[4 * (911 + 53 * j) + 2] = pair[1]  # and the second triple again in another group
    _, _, st = _stats_after(torch.from_numpy(img[None].copy()).cuda(), 2)
    ycc = matmul3_fma(img.astype(np.float64) * (1.0 / 255.0), oracle.wavelet.YCBCR_FROM_RGB,
                      post=oracle.wavelet.YCBCR_OFFSET)
    mn = _key_to_f64(st[0, 200:203].view(np.uint64))
    mx = _key_to_f64(st[0, 203:206].view(np.uint64))
    np.testing.assert_array_equal(mn.view(np.uint64), ycc.min(axis=(0, 1)).view(np.uint64))
    np.testing.assert_array_equal(mx.view(np.uint64), ycc.max(axis=(0, 1)).view(np.uint64))


@pytest.mark.parametrize("wavelet,levels,shape", [("bior1.5", None, (600, 1000)),
                                                  ("bior1.5", None, (37, 53)),
                                                  ("db1", 3, (120, 200)), ("db1", 2, (64, 96))])
def test_wavelet_fused_thresholds_match_separate(dev, monkeypatch, wavelet, levels, shape):
    """the median workgroups reduce each channel's sums of squares and set its BayesShrink
    thresholds (product) instead of the separate wl_sumsq / wl_thresh launches
    (IDN_WAVELET_FUSETHR=0, tuning build): bior1.5's partials sit on a power-of-two grid, so its
    sums -- and every output -- are bit-identical; Haar's partials add in another order (sums to
    1e-12 relative, outputs to rounding)"""
    import torch
    from idn import _lib
    x = torch.from_numpy(_stat_images(*shape)[:3] if shape != (600, 1000)
                         else np.stack([make_img(600, 1000, 21)])).cuda()
    u8a, fa, sa = _stats_after_w(x, wavelet, levels)
    monkeypatch.setenv("IDN_WAVELET_FUSETHR", "0")
    with _lib.variant("tuning"):
        u8b, fb, sb = _stats_after_w(x, wavelet, levels)
    if wavelet == "bior1.5":
        np.testing.assert_array_equal(sa.view(np.uint64), sb.view(np.uint64))
        np.testing.assert_array_equal(u8a, u8b)
        np.testing.assert_array_equal(fa, fb)
    else:
        L = levels
        fl = np.zeros(256, bool)  # the sums, medians, thresholds and half thresholds
        fl[8:8 + 9 * L + 3 + 9 * L] = True
        fl[170:197] = True
        # (NaN where a channel has no nonzero finest detail: the same in both forms)
        np.testing.assert_allclose(sa[:, fl], sb[:, fl], rtol=1e-12, atol=0, equal_nan=True)
        np.testing.assert_array_equal(sa[:, ~fl].view(np.uint64), sb[:, ~fl].view(np.uint64))
        assert np.abs(fa - fb).max() <= 1e-6
        d = u8a.astype(int) - u8b.astype(int)
        assert np.abs(d).max() <= 1 and (d != 0).mean() < 1e-4


def _stats_after_w(x, wavelet, levels):
    """denoise_wavelet on device batch x; returns (u8, f32, per-image stats blocks)"""
    import torch
    from idn import _lib, ops
    u8, f = ops.denoise_wavelet(x, wavelet, levels, out="both")
    n, h, w, _ = x.shape
    off = _lib.load().idn_wavelet_stats_offset(n, h, w, ops.WAVELETS[wavelet],
                                               -1 if levels is None else levels)
    ws = ops._WS_CACHE[(str(x.device), torch.cuda.current_stream(x.device).cuda_stream)]
    st = ws[off:off + n * 256 * 8].view(torch.float64).view(n, 256).cpu().numpy().copy()
    return u8.cpu().numpy(), f.cpu().numpy(), st


def _h3_sel(st):
    """wl_h3_* selection words per image and channel (haar3.hpp H3Sel at stats doubles 66..78):
    lo, hi, n_t, n_lo, n_c, n_r, fb"""
    return st[:, 66:78].copy().view(np.uint32).reshape(-1, 3, 8)


def _clipped(h, w, seed):
    """heavily clipped gaussian noise (config 5's var 1.0): most channels 0 or 255, many T = 0
    groups that are rounding residues in the reference's fp64 planes"""
    import oracle
    rs = np.random.RandomState(seed)
    tex = make_img(h, w, seed)
    return oracle.sk.to_u8(255 * oracle.sk.noise_gaussian(tex, rs.normal(0, 1.0, tex.shape)))


@pytest.mark.parametrize("force_fb", [False, True])
def test_haar3_two_read_path(dev, monkeypatch, force_fb):
    """round 6 Haar L = 3 (window sample, one statistics read, sigma, one synthesis read) against
    the round-4 passes on the fp64 planes (IDN_WAVELET_H3=0, IDN_WAVELET_INTSTATS=0): colour
    min / max and nonzero counts bit for bit, sums to 1e-12 relative, sigma within the analytic
    bound (bitwise where the exact full-image selection ran: IDN_WAVELET_H3FB=1 forces it for every
    channel), outputs within 1e-6 and U8 flips only on rounding boundaries.  Without forcing, the
    textured and noisy images must take the window path."""
    import torch
    from idn import _lib
    imgs = np.concatenate([_stat_images(96, 160),
                           np.stack([_clipped(96, 160, 3), _clipped(96, 160, 4)])])
    x = torch.from_numpy(imgs).cuda()
    if force_fb:
        monkeypatch.setenv("IDN_WAVELET_H3FB", "1")
        with _lib.variant("tuning"):
            u8a, fa, sa = _stats_after(x, 3)
        monkeypatch.delenv("IDN_WAVELET_H3FB")
    else:
        u8a, fa, sa = _stats_after(x, 3)
    monkeypatch.setenv("IDN_WAVELET_INTSTATS", "0")
    monkeypatch.setenv("IDN_WAVELET_H3", "0")
    with _lib.variant("tuning"):
        u8b, fb, sb = _stats_after(x, 3)
    sel = _h3_sel(sa)
    med = slice(35, 38)
    np.testing.assert_array_equal(sa[:, 200:206].view(np.uint64), sb[:, 200:206].view(np.uint64))
    np.testing.assert_array_equal(sa[:, 248:251], sb[:, 248:251])
    if force_fb:
        assert np.all(sel[:, :, 6][sa[:, 248:251] > 0] == 1)  # (no nonzero dd: no selection)
        np.testing.assert_array_equal(sa[:, med].view(np.uint64), sb[:, med].view(np.uint64))
    else:
        # textured (2), noisy (3), uniform (4), clipped (7, 8): the window path
        assert np.all(sel[[2, 3, 4, 7, 8], :, 6] == 0), sel[:, :, 6]
        rng = _key_to_f64(sb[:, 203:206].view(np.uint64)) - _key_to_f64(sb[:, 200:203].view(np.uint64))
        ok = np.abs(sa[:, med] - sb[:, med]) <= 2.1e-12 / np.maximum(rng, 1e-300)
        assert np.all(ok | (np.isnan(sa[:, med]) & np.isnan(sb[:, med])))
    live = _key_to_f64(sb[:, 203:206].view(np.uint64)) - _key_to_f64(sb[:, 200:203].view(np.uint64)) > 1e-6
    sq_a, sq_b = sa[:, 8:35].reshape(-1, 3, 9), sb[:, 8:35].reshape(-1, 3, 9)
    assert np.all((np.abs(sq_a - sq_b) <= 1e-12 * np.abs(sq_b) + 1e-300)[live])
    assert np.abs(fa - fb).max() <= 1e-6
    d = u8a.astype(int) - u8b.astype(int)
    assert np.abs(d).max() <= 1 and (d != 0).mean() < 1e-4


def test_haar3_full_size_batch_vs_oracle(dev):
    """the bench's shape: a batch of 600x1000 images (textured, noisy, clipped) through the
    round-6 Haar L = 3 path, each image against the oracle within 1e-5 (U8 flips only at rounding
    boundaries), and the u8-only launch (dword stores) equal to the u8 + f32 launch byte for byte"""
    import torch
    import idn
    import oracle
    imgs = np.stack([make_img(600, 1000, 41),
                     oracle.sk.to_u8(255 * oracle.sk.noise_gaussian(
                         make_img(600, 1000, 42), np.random.RandomState(42).normal(0, 0.3, (600, 1000, 3)))),
                     _clipped(600, 1000, 43)])
    x = torch.from_numpy(imgs).cuda()
    u8, f = idn.ops.denoise_wavelet(x, "db1", 3, out="both")
    u8only = idn.ops.denoise_wavelet(x, "db1", 3)
    assert torch.equal(u8, u8only)
    f, u8 = f.cpu().numpy().astype(np.float64), u8.cpu().numpy()
    for i in range(len(imgs)):
        ref = oracle.wavelet.denoise_wavelet(imgs[i], "db1", 3)
        assert np.abs(f[i] - ref).max() <= TOL, i
        check_u8(u8[i], ref, oracle.sk.to_u8(255 * ref))
