"""GPU parity of the reference's own additive noises (uniform / gamma / rayleigh / brownian,
lib/model/test.py:767-1572): replay mode vs the scipy/numpy fixtures, Philox-mode statistics."""
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"


@pytest.fixture(scope="module")
def gold():
    g = np.load(GOLD / "golden.npz", allow_pickle=False)
    m = json.loads((GOLD / "golden.json").read_text())
    return g, m


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _run(img, mode, level, field=None, **kw):
    import torch
    import idn
    x = torch.from_numpy(np.ascontiguousarray(img)).cuda()
    rp = None if field is None else torch.from_numpy(np.ascontiguousarray(field[None] if field.ndim == 3 else field)).cuda()
    u8, f = idn.ops.noise_add(x, mode, level, replay=rp, out="both", **kw)
    return u8.cpu().numpy(), f.cpu().numpy()


def test_additive_replay_vs_fixtures(dev, gold):
    from test_oracle import additive_draws
    g, m = gold
    for case in m["additive"]:
        img = g["in_" + case["input"]]
        field = additive_draws(case["mode"], case["seed"], img)
        u8, f = _run(img, case["mode"], case["level"], field)
        if case["mode"] == "brownian":
            # fp64 block scan vs np.cumsum's sequential order: rounding only
            assert (u8 != g[case["key"] + "_u8"]).mean() < 1e-3, case
            from oracle import sk
            ref = sk.brownian_walk(field.reshape(-1)[1:], case["level"]).reshape(img.shape)
            assert np.abs(f - ref).max() <= 1e-12 * max(1.0, np.abs(ref).max()), case
        else:
            assert np.array_equal(u8, g[case["key"] + "_u8"]), case
            assert sha(f.astype(np.float64)) == case["sha_f64"], case


def test_brownian_full_size_replay(dev):
    from oracle import sk
    from test_oracle import make_img
    img = make_img(600, 1000, 5)
    rs = np.random.RandomState(77)
    z = rs.normal(size=img.size - 1)
    field = np.concatenate([[0.0], z]).reshape(img.shape)
    for dt in (0.9, 0.009):
        u8, walk = _run(img, "brownian", dt, field)
        ref_walk = sk.brownian_walk(z, dt).reshape(img.shape)
        assert np.abs(walk - ref_walk).max() < 1e-9
        ref = sk.noise_brownian(img, z, dt)
        assert (u8 != ref).mean() < 1e-5


@pytest.mark.parametrize("mode,level,mean,var", [
    ("uniform", 0.6, 0.3, 0.36 / 12),
    ("gamma", 0.1, 1.99 * 0.1, 1.99 * 0.01),
    ("rayleigh", 0.2, 0.2 * np.sqrt(np.pi / 2), (4 - np.pi) / 2 * 0.04),
])
def test_additive_philox_moments(dev, mode, level, mean, var):
    img = np.full((2, 300, 500, 3), 51, np.uint8)  # 51/255 = 0.2 exactly representable? no: any
    u8, f = _run(img, mode, level, seed=13, offset=2)
    d = (f - img.astype(np.float64) * (1.0 / 255.0)).reshape(-1)
    assert abs(d.mean() - mean) < 3e-3 * max(1.0, mean / 0.1)
    assert abs(d.var() - var) / var < 1e-2
    assert np.array_equal(u8, __import__("oracle").sk.to_u8(255 * f))
    if mode == "uniform":
        assert d.min() >= 0.0 and d.max() < level


def test_brownian_philox_increments(dev):
    img = np.zeros((1, 200, 300, 3), np.uint8)
    u8, walk = _run(img, "brownian", 0.09, seed=3)
    b = walk.reshape(-1)
    assert b[0] == 0.0
    inc = np.diff(b)
    assert abs(inc.mean()) < 3e-3 and abs(inc.var() / 0.09 - 1) < 1e-2
    from oracle import sk
    assert np.array_equal(u8.reshape(-1), np.minimum(sk.to_u8(b * 255), 255))


@pytest.mark.parametrize("mode", ["uniform", "gamma", "rayleigh", "brownian"])
def test_additive_offset_is_image_id(dev, mode):
    import torch
    import idn
    from test_oracle import make_img
    imgs = np.stack([make_img(30, 50, s) for s in range(3)])
    x = torch.from_numpy(imgs).cuda()
    full = idn.ops.noise_add(x, mode, 0.2, seed=5, offset=10).cpu().numpy()
    for i in range(3):
        one = idn.ops.noise_add(x[i:i + 1], mode, 0.2, seed=5, offset=10 + i).cpu().numpy()
        assert np.array_equal(full[i], one[0])


@pytest.mark.parametrize("mode", ["uniform", "gamma", "rayleigh", "brownian"])
def test_additive_image_ids_match_offsets(dev, mode):
    """one launch over arbitrary image ids == per-image offset launches"""
    import torch
    import idn
    from test_oracle import make_img
    imgs = np.stack([make_img(24, 40, s) for s in range(3)])
    x = torch.from_numpy(imgs).cuda()
    ids = [9, 2, 40]
    level = {"uniform": 0.2, "gamma": 0.05, "rayleigh": 0.1, "brownian": 1e-6}[mode]
    u8 = idn.ops.noise_add(x, mode, level, seed=2, image_ids=ids).cpu().numpy()
    for k, i in enumerate(ids):
        one = idn.ops.noise_add(x[k:k + 1], mode, level, seed=2, offset=i).cpu().numpy()
        assert np.array_equal(u8[k], one[0])
