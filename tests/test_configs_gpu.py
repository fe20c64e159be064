"""End-to-end parity of the multi-GPU BASELINE workloads as bench.py runs them, at 600x1000.

Config 5 (BASELINE.json configs[4]): a seeded mixed-noise batch, each type noised in place through
slot-addressed launches (bench.py `_pipeline("cfg5")`; the reference's mix dispatcher
minibatch.py:1518-1574 picks one noise per image), then the 3-level Haar BayesShrink wavelet
(minibatch_before_curvelet.py:85-87).  Checked: the slot-addressed batch equals per-image
random_noise / periodic / copy calls byte for byte, and the wavelet output is within 1e-5 of the
oracle's denoise_wavelet on the same noised bytes (U8 differences only at integer boundaries).

Config 4 (configs[3]): Philox speckle var 1.0 then cv2.bilateralFilter(9, 75, 75)
(minibatch.py:1658-1663): within 1 LSB of the oracle's bilateral on the same noised bytes, the
1-LSB cases on rounding boundaries only."""
import sys
from pathlib import Path

import numpy as np
import pytest

from conftest import textured

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent
TOL = 1e-5


def _bench():
    if str(ROOT) not in sys.path:
        sys.path.insert(0, str(ROOT))
    import bench
    return bench


def test_config5_mixed_noise_haar3_end_to_end(dev):
    import torch
    import idn
    import oracle
    bench = _bench()
    n = 12
    x = torch.from_numpy(textured(n, 600, 1000, seed=31)).cuda()
    y = torch.empty_like(x)
    step = bench._pipeline("cfg5")
    step(idn, x, y)
    torch.cuda.synchronize()
    groups = step.state["groups"]
    t = step.state["t"]
    kinds = {i: k for k, (v, _) in groups.items() for i in v}
    assert len(kinds) == n and len(groups) >= 4, groups.keys()
    # 1) the slot-addressed noise == per-image calls with image id = batch position
    ops = idn.ops
    for i in range(n):
        xi, k = x[i:i + 1], kinds[i]
        if k == "original":
            ref = xi
        elif k == "periodic":
            ref = ops.periodic_noise(xi, 100.0)
        elif k == "s&p":
            ref = ops.random_noise(xi, "s&p", amount=0.4, seed=3, image_ids=[i], out="u8")
        elif k == "poisson":
            ref = ops.random_noise(xi, "poisson", seed=3, image_ids=[i], out="u8")
        else:
            ref = ops.random_noise(xi, k, var=1.0, seed=3, image_ids=[i], out="u8")
        assert torch.equal(t[i], ref[0]), (i, k)
    # 2) the Haar L=3 output vs the oracle on the same noised bytes (one image of every type)
    u8b, fb = ops.denoise_wavelet(t, "db1", 3, out="both")
    assert torch.equal(u8b, y)
    tn, fbn, yn = t.cpu().numpy(), fb.cpu().numpy().astype(np.float64), y.cpu().numpy()
    firsts = sorted(v[0] for v, _ in groups.values())
    for i in firsts:
        ref = oracle.wavelet.denoise_wavelet(tn[i], "db1", 3)
        assert np.abs(fbn[i] - ref).max() <= TOL, (i, kinds[i])
        d = yn[i].astype(int) - oracle.sk.to_u8(255 * ref).astype(int)
        assert np.abs(d).max() <= 1
        near = np.abs(255 * ref - np.round(255 * ref)) < 255 * TOL + 1e-9
        assert np.all(near[d != 0]), (i, kinds[i])


def test_config4_speckle_bilateral_end_to_end(dev):
    import torch
    import idn
    import oracle
    bench = _bench()
    n = 3
    x = torch.from_numpy(textured(n, 600, 1000, seed=41)).cuda()
    y = torch.empty_like(x)
    step = bench._pipeline("cfg4")
    step(idn, x, y)
    torch.cuda.synchronize()
    t = step.state["t"]
    ref_t = idn.ops.random_noise(x, "speckle", var=1.0, seed=3, out="u8")
    assert torch.equal(t, ref_t)
    tn, yn = t.cpu().numpy(), y.cpu().numpy()
    ref = oracle.cv.bilateral_filter(tn, 9, 75.0, 75.0)
    d = np.abs(yn.astype(int) - ref.astype(int))
    assert d.max() <= 1
    pre = oracle.cv.bilateral_prefilter_f32(tn, 9, 75.0, 75.0)
    frac = np.abs(pre - np.floor(pre) - 0.5)
    assert np.all(frac[d > 0] < 1e-3)
    assert (d > 0).mean() < 1e-3
