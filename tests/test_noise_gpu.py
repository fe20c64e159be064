"""GPU parity of the noise generators, periodic pattern and blob epilogue.

Replay mode (numpy's own random field fed to the kernel) must reproduce skimage's random_noise
bit-exactly (u8 and float64), checked against the golden fixtures (tests/golden) and the oracle.
Philox mode is checked statistically: moments / KS distance of the generated noise and the
s&p flip rates, at BASELINE's full 600x1000 size.
"""
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

from test_oracle import make_img, oracle_noise, replay_field

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD / "golden.npz", allow_pickle=False), json.loads((GOLD / "golden.json").read_text())


MODE = {"gaussian": "gaussian", "speckle": "speckle", "s&p": "s&p", "poisson": "poisson"}


def gpu_noise(img, case, field):
    import torch
    import idn
    x = torch.from_numpy(img).cuda()
    kw = dict(case["kw"])
    rp = torch.from_numpy(np.ascontiguousarray(field, np.float64)).cuda()
    u8, f64 = idn.ops.random_noise(x, case["mode"], replay=rp, out="both", **kw)
    torch.cuda.synchronize()
    return u8.cpu().numpy(), f64.cpu().numpy()


def test_replay_bitexact_small(dev, gold):
    g, m = gold
    for case in m["noise"]:
        if case["key"] is None:
            continue
        img = g["in_" + case["input"]]
        field = replay_field(case["mode"], case["kw"], case["seed"], img)
        u8, f64 = gpu_noise(img, case, field)
        assert sha(f64) == case["sha_f64"], case
        assert np.array_equal(u8, g[case["key"] + "_u8"]), case


def test_replay_bitexact_full_size(dev, gold):
    _, m = gold
    big = make_img(600, 1000, 5)
    for case in m["noise"]:
        if case["key"] is not None:
            continue
        field = replay_field(case["mode"], case["kw"], case["seed"], big)
        u8, f64 = gpu_noise(big, case, field)
        assert sha(f64) == case["sha_f64"], case
        assert sha(u8) == case["sha_u8"], case


def test_replay_batch_matches_per_image(dev):
    """a batch of 3 images with per-image fields == three single-image calls (oracle)"""
    import torch
    import idn
    import oracle
    imgs = np.stack([make_img(30, 44, s) for s in (1, 2, 3)])
    for mode, kw in (("gaussian", {"var": 1.5}), ("speckle", {"var": 1.0}),
                     ("s&p", {"amount": 0.2}), ("poisson", {})):
        fields = [replay_field(mode, dict(kw, var=kw.get("var", 0)), 77 + i, imgs[i]) for i in range(3)]
        if mode == "s&p":
            field = np.stack([np.stack([f[0] for f in fields]), np.stack([f[1] for f in fields])])
        else:
            field = np.stack(fields)
        x = torch.from_numpy(imgs).cuda()
        u8, f64 = idn.ops.random_noise(x, mode, replay=torch.from_numpy(field).cuda(), out="both", **kw)
        for i in range(3):
            ref = oracle_noise(mode, kw, imgs[i], fields[i])
            assert np.array_equal(f64[i].cpu().numpy(), ref)
            assert np.array_equal(u8[i].cpu().numpy(), oracle.sk.to_u8(255 * ref))


def _philox(img, mode, **kw):
    import torch
    import idn
    x = torch.from_numpy(img).cuda()
    u8, f64 = idn.ops.random_noise(x, mode, out="both", **kw)
    return u8.cpu().numpy(), f64.cpu().numpy()


def test_philox_gaussian_statistics(dev):
    """unclipped region: out - x ~ N(0, sqrt(var)); KS distance against the normal CDF"""
    from math import erf, sqrt
    img = np.full((1, 600, 1000, 3), 128, np.uint8)
    var = 0.0025  # small so clipping never triggers around 0.5
    _, f64 = _philox(img, "gaussian", var=var, seed=3)
    z = np.sort(((f64 - 128 / 255.0) / sqrt(var)).reshape(-1))
    assert abs(z.mean()) < 5e-3 and abs(z.std() - 1) < 5e-3
    cdf = 0.5 * (1 + np.vectorize(erf)(z[:: 97] / sqrt(2)))
    emp = (np.arange(z.size)[::97] + 0.5) / z.size
    assert np.abs(cdf - emp).max() < 3e-3


def test_philox_speckle_and_determinism(dev):
    img = make_img(600, 1000, 5)[None]
    a8, a = _philox(img, "speckle", var=0.5, seed=11, offset=3)
    b8, b = _philox(img, "speckle", var=0.5, seed=11, offset=3)
    c8, _ = _philox(img, "speckle", var=0.5, seed=12, offset=3)
    assert np.array_equal(a, b) and np.array_equal(a8, b8)
    assert (a8 != c8).mean() > 0.5
    # small variance, mid-range x: no clipping within 5 sigma, so n = (out - x) / x is unbiased
    _, a = _philox(img, "speckle", var=0.0025, seed=11, offset=3)
    x = img.astype(np.float64) * (1.0 / 255.0)
    m = (x > 0.1) & (x < 0.75)
    n = (a[m] - x[m]) / x[m]
    assert abs(n.mean()) < 5e-4 and abs(n.std() - 0.05) < 5e-4


def test_philox_offset_is_image_id(dev):
    """image i of a batch with offset o == image 0 of a single call with offset o + i"""
    import torch
    import idn
    imgs = np.stack([make_img(40, 60, s) for s in range(4)])
    x = torch.from_numpy(imgs).cuda()
    full = idn.ops.random_noise(x, "gaussian", var=1.0, seed=5, offset=10).cpu().numpy()
    for i in range(4):
        one = idn.ops.random_noise(x[i:i + 1], "gaussian", var=1.0, seed=5, offset=10 + i).cpu().numpy()
        assert np.array_equal(full[i], one[0])


def test_philox_sap_rates(dev):
    img = make_img(600, 1000, 5)[None]
    for amount in (0.2, 0.4, 0.8):
        u8, f64 = _philox(img, "s&p", amount=amount, seed=7)
        x = img.astype(np.float64) * (1.0 / 255.0)  # img_as_float
        salt = (f64 == 1.0) & (x != 1.0)
        pep = (f64 == 0.0) & (x != 0.0)
        keep = f64 == x
        inner = (x > 0) & (x < 1)  # flips on already-black / white pixels are invisible
        assert abs(salt[inner].mean() - amount / 2) < 3e-3
        assert abs(pep[inner].mean() - amount / 2) < 3e-3
        assert np.all(salt | pep | keep)
        assert np.all(u8[salt] == 255) and np.all(u8[pep] == 0)


def test_philox_poisson_statistics(dev):
    import oracle
    rs = np.random.RandomState(0)
    img = rs.randint(0, 256, (1, 600, 1000, 3)).astype(np.uint8)
    vals = oracle.sk.poisson_vals(img[0])
    assert vals == 256
    _, f64 = _philox(img, "poisson", seed=9)
    lam = img.astype(np.float64) / 255 * vals
    k = f64 * vals
    assert np.all(k == np.round(k))
    for lo, hi in ((0.5, 3), (3, 10), (10, 30), (100, 200)):
        sel = (lam >= lo) & (lam < hi) & (f64 < 1)
        r = (k[sel] - lam[sel])
        assert abs(r.mean()) < 0.02 * np.sqrt(lam[sel].mean())
        assert abs((r ** 2).mean() / lam[sel].mean() - 1) < 0.02


def test_philox_poisson_distribution(dev):
    """the inversion sampler's law: for several lambdas the empirical CDF of the counts matches
    the exact Poisson CDF (scipy.stats) within the KS 99.9 % bound 1.95 / sqrt(n)"""
    from scipy.stats import poisson
    # every u8 value equally often -> vals = 256, lambda = v / 255 * 256
    flat = np.arange(8 * 240 * 400 * 3) % 256
    img = flat.astype(np.uint8).reshape(8, 240, 400, 3)
    _, f64 = _philox(img, "poisson", seed=21)
    k = np.round(f64 * 256).astype(np.int64)
    for v in (1, 4, 10, 40, 128, 200):
        lam = v / 255 * 256
        sel = (img == v) & (f64 < 1)  # clip(k / 256) saturates k >= 256
        ks = k[sel]
        n = int((img == v).sum())
        emp = np.bincount(ks, minlength=256)[:256].cumsum() / n
        ref = poisson.cdf(np.arange(256), lam)
        assert np.max(np.abs(emp - ref)) < 1.95 / np.sqrt(n), v


def test_poisson_vals_per_image(dev):
    """vals = 2**ceil(log2(#unique)) per image: image with 3 distinct values -> vals 4"""
    import torch
    import idn
    a = np.zeros((2, 8, 16, 3), np.uint8)
    a[0, :, :8] = 10
    a[0, :, 8:] = 200
    a[0, 0, 0, 0] = 77           # 4 distinct values incl. 0? -> {10, 200, 77} + none = 3 -> 4
    a[1] = np.arange(8 * 16 * 3).reshape(8, 16, 3) % 256  # 256 distinct -> 256 (and 0 present)
    lam = np.zeros(a.shape)
    x = torch.from_numpy(a).cuda()
    rp = torch.zeros(a.shape, dtype=torch.float64, device="cuda")
    rp[0] = 3.0
    rp[1] = 3.0
    _, f64 = idn.ops.random_noise(x, "poisson", replay=rp, out="both")
    f = f64.cpu().numpy()
    assert np.allclose(f[0], 3.0 / 4) and np.allclose(f[1], 3.0 / 256)
    del lam


def test_periodic_pattern_gpu(dev, gold):
    import oracle
    import idn
    _, m = gold
    for case in m["periodic"]:
        pat = idn.ops.periodic_pattern(case["h"], case["w"], 3, case["amp"]).cpu().numpy()
        ref = oracle.sk.periodic_pattern(case["h"], case["w"], 3, case["amp"])
        diff = np.flatnonzero(pat.reshape(-1) != ref.reshape(-1))
        assert set(diff.tolist()) <= set(case["near_int_idx"]), (case["amp"], diff[:10])


def test_periodic_noise_add(dev):
    import torch
    import idn
    import oracle
    img = make_img(600, 1000, 5)
    x = torch.from_numpy(np.stack([img, img[::-1].copy()])).cuda()
    got = idn.ops.periodic_noise(x, 100.0).cpu().numpy()
    pat = idn.ops.periodic_pattern(600, 1000, 3, 100.0).cpu().numpy()
    assert np.array_equal(got[0], oracle.sk.add_saturate(img, pat))
    assert np.array_equal(got[1], oracle.sk.add_saturate(img[::-1], pat))


@pytest.mark.parametrize("flip", [False, True])
def test_blob_bitexact(dev, flip):
    import torch
    import idn
    import oracle
    imgs = np.stack([make_img(600, 1000, s) for s in (1, 2)])
    x = torch.from_numpy(imgs).cuda()
    got = idn.ops.blob(x, flip=flip).cpu().numpy()
    ref = oracle.sk.blob_f32(list(imgs), flip=flip)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    padded = idn.ops.blob(x[:1, :500, :700], out_hw=(600, 1000)).cpu().numpy()
    refp = oracle.sk.blob_f32([imgs[0, :500, :700], np.zeros((600, 1000, 3), np.uint8)])[:1]
    refp[0, 500:] = 0
    refp[0, :, 700:] = 0
    assert np.array_equal(padded, refp)


KINDS = {"gaussian": 0, "speckle": 1, "s&p": 2, "poisson": 3}


def noise_padded(imgs, mode, kw, seed, offset, out="u8", pad=16):
    """idn_noise_u8 through the C-ABI on rows padded to w*c + pad bytes: the element kernels
    (strided rows) instead of the flat ones"""
    import torch
    from idn import _lib
    n, h, w, c = imgs.shape
    rs = w * c + pad
    buf = np.zeros((n, h, rs), np.uint8)
    buf[:, :, :w * c] = imgs.reshape(n, h, w * c)
    x = torch.from_numpy(buf).cuda()
    y8 = torch.zeros_like(x) if out in ("u8", "both") else None
    y64 = torch.zeros((n, h, w, c), dtype=torch.float64, device="cuda") if out in ("f64", "both") else None
    kind = KINDS[mode]
    p0, p1 = ((kw.get("amount", 0.05), 0.5) if kind == 2 else (0.0, kw.get("var", 0.0)))
    lib = _lib.load()
    wsb = lib.idn_noise_workspace_size(kind, n)
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device="cuda")
    rc = lib.idn_noise_u8(x.data_ptr(), y8.data_ptr() if y8 is not None else None,
                          y64.data_ptr() if y64 is not None else None, n, h, w, c, rs, kind,
                          float(p0), float(p1), seed, offset, None, ws.data_ptr(), wsb,
                          torch.cuda.current_stream().cuda_stream)
    _lib.check(rc, "idn_noise_u8")
    torch.cuda.synchronize()
    u8 = y8.cpu().numpy()[:, :, :w * c].reshape(n, h, w, c) if y8 is not None else None
    f64 = y64.cpu().numpy() if y64 is not None else None
    return u8, f64


@pytest.mark.parametrize("mode,kw", [("gaussian", {"var": 0.1}), ("speckle", {"var": 1.0}),
                                     ("s&p", {"amount": 0.4}), ("poisson", {})])
def test_philox_forms_consistent(dev, mode, kw):
    """flat (compact rows, 16 elements / lane) and element (strided rows) kernels draw the same
    stream: identical u8-only outputs, identical float64 outputs; out="both" gives
    U8 == trunc(255 * f64) exactly; deterministic and batch-split invariant."""
    import oracle
    import torch
    import idn
    imgs = np.stack([make_img(120, 200, s) for s in range(3)])
    x = torch.from_numpy(imgs).cuda()
    u8 = idn.ops.random_noise(x, mode, seed=4, offset=7, out="u8", **kw).cpu().numpy()
    b8, f64 = idn.ops.random_noise(x, mode, seed=4, offset=7, out="both", **kw)
    b8, f64 = b8.cpu().numpy(), f64.cpu().numpy()
    assert np.array_equal(b8, oracle.sk.to_u8(255 * f64))
    p8, _ = noise_padded(imgs, mode, kw, 4, 7, out="u8")
    assert np.array_equal(p8, u8)
    q8, q64 = noise_padded(imgs, mode, kw, 4, 7, out="both")
    assert np.array_equal(q64, f64) and np.array_equal(q8, b8)
    one8 = idn.ops.random_noise(x[1:2], mode, seed=4, offset=8, **kw).cpu().numpy()
    assert np.array_equal(one8[0], u8[1])
    _, one64 = idn.ops.random_noise(x[1:2], mode, seed=4, offset=8, out="both", **kw)
    assert np.array_equal(one64[0].cpu().numpy(), f64[1])
    if mode in ("s&p", "poisson"):  # one stream: the u8-only and float64 calls draw the same
        assert np.array_equal(u8, b8)


def _normal_cdf(t):
    from scipy.special import erf
    return 0.5 * (1.0 + erf(np.asarray(t, np.float64) / np.sqrt(2.0)))


def u8_law(mode, sd, v):
    """P(U8 output = k), k = 0..255, for input byte v: gaussian floor(clip(v + 255 sd z)),
    speckle floor(clip(v (1 + sd z))) on the 0..255 scale (255 * clip(x + n, 0, 1) truncated;
    x = v / 255)"""
    k = np.arange(257, dtype=np.float64)
    if mode == "gaussian":
        edges = _normal_cdf((k - v) / (255.0 * sd))  # P(v + 255 sd z < k)
    else:
        if v == 0:
            p = np.zeros(256)
            p[0] = 1.0
            return p
        edges = _normal_cdf((k / v - 1.0) / sd)
    p = np.diff(edges[:256])  # P(k <= out < k + 1), k = 0..254
    p = np.concatenate([p, [1.0 - edges[255]]])  # out >= 255
    p[0] += edges[0]  # out < 0 clips to 0
    return p


@pytest.mark.parametrize("mode,var", [("gaussian", 0.1), ("gaussian", 1.0), ("gaussian", 1.5),
                                      ("speckle", 0.5), ("speckle", 1.0), ("speckle", 2.0)])
def test_philox_u8_law_chi_square(dev, mode, var):
    """The u8 stream's output law at the reference's levels (README.md:90-100; test.py:193-307,
    476-590), full 600x1000 textured images: for every input value v, the histogram of U8 outputs
    against the exact P(U8 = k) from the normal CDF.  Bins pooled to expected >= 5 per v; the
    summed statistic over all v must not be significant at the 1e-4 level (fixed seeds)."""
    import torch
    import idn
    from scipy.stats import chi2
    imgs = np.stack([make_img(600, 1000, s) for s in (1, 2, 3)])
    x = torch.from_numpy(imgs).cuda()
    sd = var ** 0.5
    stat, dof = 0.0, 0
    for seed in (3, 4):
        u8 = idn.ops.random_noise(x, mode, var=var, seed=seed, out="u8").cpu().numpy()
        vin = imgs.reshape(-1).astype(np.int64)
        vout = u8.reshape(-1).astype(np.int64)
        counts = np.bincount(vin * 256 + vout, minlength=256 * 256).reshape(256, 256)
        for v in range(256):
            nv = counts[v].sum()
            if nv < 200:
                continue
            exp = u8_law(mode, sd, v) * nv
            obs = counts[v].astype(np.float64)
            # pool adjacent bins left to right until each pooled bin expects >= 5
            pe, po, ce, co = [], [], 0.0, 0.0
            for e_, o_ in zip(exp, obs):
                ce += e_
                co += o_
                if ce >= 5:
                    pe.append(ce)
                    po.append(co)
                    ce = co = 0.0
            if pe:
                pe[-1] += ce
                po[-1] += co
            if len(pe) < 2:
                assert abs(po[0] - pe[0]) < 1e-6 * nv + 1e-9, (v, po, pe)
                continue
            pe, po = np.array(pe), np.array(po)
            stat += float(((po - pe) ** 2 / pe).sum())
            dof += len(pe) - 1
    p = chi2.sf(stat, dof)
    assert p > 1e-4, (mode, var, stat, dof, p)


def test_philox_f64_law_chi_square(dev):
    """the float64 stream's U8 (= trunc(255 * out)) follows the same law"""
    import torch
    import idn
    from scipy.stats import chi2
    imgs = np.stack([make_img(600, 1000, s) for s in (1, 2)])
    x = torch.from_numpy(imgs).cuda()
    for mode, var in (("gaussian", 1.0), ("speckle", 0.5)):
        u8, _ = idn.ops.random_noise(x, mode, var=var, seed=5, out="both")
        u8 = u8.cpu().numpy()
        counts = np.bincount(imgs.reshape(-1).astype(np.int64) * 256 + u8.reshape(-1),
                             minlength=65536).reshape(256, 256)
        stat, dof = 0.0, 0
        for v in range(0, 256, 3):
            nv = counts[v].sum()
            if nv < 500 or (mode == "speckle" and v == 0):
                continue
            exp = u8_law(mode, var ** 0.5, v) * nv
            keep = exp >= 5
            pe = np.concatenate([exp[keep], [exp[~keep].sum()]])
            po = np.concatenate([counts[v][keep], [counts[v][~keep].sum()]]).astype(np.float64)
            if pe[-1] < 5:
                pe[-2] += pe[-1]
                po[-2] += po[-1]
                pe, po = pe[:-1], po[:-1]
            stat += float(((po - pe) ** 2 / pe).sum())
            dof += len(pe) - 1
        assert chi2.sf(stat, dof) > 1e-4, (mode, stat, dof)


def test_philox_u8_tail_reaches_past_the_16_bit_grid(dev):
    """the refined extreme cell: |z| beyond sqrt(2 ln 2^16) = 4.71 occurs (0 without the
    refinement).  Speckle var 1e-4 on v = 200: U8 = floor(200 (1 + 0.01 z)) = floor(200 + 2 z)."""
    import torch
    import idn
    img = np.full((8, 600, 1000, 3), 200, np.uint8)
    x = torch.from_numpy(img).cuda()
    u8 = idn.ops.random_noise(x, "speckle", var=1e-4, seed=9, out="u8").cpu().numpy().astype(int)
    # floor(200 + 2 z) >= 210 iff z >= 5; <= 189 iff z < -5: P(|z| > 5) = 5.7e-7, ~8 of 14.4 M
    beyond = int(((u8 >= 210) | (u8 <= 189)).sum())
    assert 0 < beyond < 40, beyond
    assert np.abs(u8 - 200).max() <= 14  # |z| <= 6.66


def test_poisson_levels_staged(dev):
    """every vals level's guide + threshold window fits the flat kernel's LDS block, so its draws
    take the LDS path (a level over capacity would silently fall back to bisecting the rows)"""
    import ctypes
    import torch
    import idn
    from idn import _lib
    lib = _lib.load()
    ntab = (ctypes.c_uint32 * 9)()
    cap = (ctypes.c_uint32 * 1)()
    _lib.check(lib.idn_poisson_levels(ntab, cap, torch.cuda.current_stream().cuda_stream),
               "idn_poisson_levels")
    assert all(0 < t <= cap[0] for t in ntab), (list(ntab), cap[0])
    assert ntab[8] > ntab[0]  # vals = 256: the widest windows


def test_poisson_flat_matches_element_kernel(dev):
    """the flat Poisson kernel (16 elements per thread, LDS bucket tables) and the element kernel
    (strided rows) take the same uniforms, buckets and walk: identical outputs, over images of
    several vals (3, 16 and 256 distinct values)"""
    import torch
    import idn
    imgs = np.stack([make_img(48, 64, s) for s in (1, 2, 3, 4)])
    imgs[0, :8] //= 16  # dark rows: small lambda
    imgs[2] = (imgs[2] // 86) * 86  # 3 distinct values -> vals 4
    imgs[3] = (imgs[3] // 16) * 16  # 16 distinct values -> vals 16
    x = torch.from_numpy(imgs).cuda()
    u8, f64 = idn.ops.random_noise(x, "poisson", seed=5, offset=3, out="both")
    p8, p64 = noise_padded(imgs, "poisson", {}, 5, 3, out="both")
    assert np.array_equal(u8.cpu().numpy(), p8)
    assert np.array_equal(f64.cpu().numpy(), p64)


@pytest.mark.parametrize("mode,kw", [("gaussian", {"var": 0.1}), ("s&p", {"amount": 0.4}),
                                     ("poisson", {}), ("speckle", {"var": 1.0})])
def test_image_ids_match_per_image_offsets(dev, mode, kw):
    """one launch over arbitrary image ids draws exactly what per-image offset launches draw"""
    import torch
    import idn
    imgs = np.stack([make_img(40, 64, s) for s in range(4)])
    x = torch.from_numpy(imgs).cuda()
    ids = [17, 3, 250, 4]
    u8, f64 = idn.ops.random_noise(x, mode, seed=6, image_ids=ids, out="both", **kw)
    for k, i in enumerate(ids):
        one8, one64 = idn.ops.random_noise(x[k:k + 1], mode, seed=6, offset=i, out="both", **kw)
        assert np.array_equal(u8[k].cpu().numpy(), one8[0].cpu().numpy())
        assert np.array_equal(f64[k].cpu().numpy(), one64[0].cpu().numpy())
    # the same ids as an int64 tensor already on the device (used as is, no host round trip)
    dev8 = idn.ops.random_noise(x, mode, seed=6, image_ids=torch.tensor(ids, device="cuda"),
                                out="u8", **kw)
    assert torch.equal(dev8, idn.ops.random_noise(x, mode, seed=6, image_ids=ids, out="u8", **kw))
    with pytest.raises(ValueError):
        idn.ops.random_noise(x, mode, seed=6, image_ids=torch.tensor(ids[:3], device="cuda"), **kw)


@pytest.mark.parametrize("mode,kw", [("gaussian", {"var": 1.0}), ("speckle", {"var": 1.0}),
                                     ("s&p", {"amount": 0.4}), ("poisson", {}),
                                     ("periodic", {}), ("original", {})])
def test_slots_match_gather_noise_scatter(dev, mode, kw):
    """slot-addressed noise (idn_noise_slots_u8 / idn_add_pattern_slots_u8 / idn_copy_slots_u8)
    writes exactly what gather -> per-group launch with image ids -> scatter writes, and leaves
    every other image of the output untouched"""
    import torch
    import idn
    imgs = np.stack([make_img(32, 48, s) for s in range(7)])
    x = torch.from_numpy(imgs).cuda()
    idx = torch.tensor([5, 1, 3], dtype=torch.int64, device="cuda")
    ops = idn.ops
    got = torch.full_like(x, 77)
    ref = torch.full_like(x, 77)
    xs = x.index_select(0, idx)
    if mode == "original":
        ops.copy_slots(x, got, idx)
        ys = xs
    elif mode == "periodic":
        ops.periodic_noise(x, 100.0, out=got, slots=idx)
        ys = ops.periodic_noise(xs, 100.0)
    else:
        ops.random_noise(x, mode, seed=4, image_ids=idx, slots=idx, out_u8=got, **kw)
        ys = ops.random_noise(xs, mode, seed=4, image_ids=idx, out="u8", **kw)
    ref.index_copy_(0, idx, ys)
    assert torch.equal(got, ref)
