"""The reference's live test path at its real size, and batch invariance of the wavelet denoiser.

lib/model/test.py:1678-1684: test_v0 `gaussian*` draws var from {0.1, 1.0, 1.5} and returns
random_noise(img, 'gaussian', var) as float64; the only live post hook (test.py:1802-1810) then
runs denoise_wavelet(im, BayesShrink, soft, wavelet='bior1.5', multichannel, convert2ycbcr) on that
float64 image -- at 600x1000 three levels of bior1.5 on f64 input -- and casts (255 * x) to uint8.

Tolerance (north star): the float result within 1e-5 of the oracle before the cast; a U8 value may
differ only where 255 * x lies within 255e-5 of an integer (the cast is discontinuous there).
"""
import json
import random

import numpy as np
import pytest

from conftest import textured

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _plan_with_var(spec, var):
    """a test_v0 plan of `spec` whose random.choice drew gaussian var `var` (and its rng seed)"""
    from idn import noise_spec as ns
    for s in range(1000):
        p = ns.plan(spec, "test_v0", random.Random(s))
        if p.steps[0].args[0] == var:
            return p
    raise AssertionError(f"no seed draws var {var}")


@pytest.mark.parametrize("var", [0.1, 1.0, 1.5])
def test_live_gaussian_wavelet_full_size(dev, var):
    import torch
    import oracle
    from idn import ops
    from idn.pipeline import Preprocessor
    from test_wavelet_gpu import check_u8

    spec = f"gaussian_wavelet_var{var}"
    plan = _plan_with_var(spec, var)
    assert [s.op for s in plan.steps] == ["gaussian", "wavelet"] and plan.steps[1].args == ("bior1.5", None)
    img = textured(1, 600, 1000, seed=int(var * 10) + 1)[0]

    # oracle: skimage random_noise with numpy's draws, then the 0.14.2 denoise_wavelet on float64
    np.random.seed(1234)
    field = np.random.normal(0.0, var ** 0.5, img.shape)
    noisy = oracle.sk.noise_gaussian(img, field)
    ref_f = oracle.wavelet.denoise_wavelet(noisy, "bior1.5", None)
    ref_u8 = oracle.sk.to_u8(255 * ref_f)

    # the drop-in surface: plan -> Preprocessor (numpy stream replayed on the device) -> U8
    pre = Preprocessor(spec, "test_v0", noise_rng="numpy")
    np.random.seed(1234)
    outs, _ = pre(torch.from_numpy(img[None]).cuda(), image_ids=[0], plans=[plan])
    got_u8 = outs[0].cpu().numpy()

    # the same two steps through ops, keeping the float64 noisy image and the float result
    x = torch.from_numpy(img[None]).cuda()
    f64 = ops.random_noise(x, "gaussian", var=var, replay=torch.from_numpy(field[None]).cuda(),
                           out="f64")
    np.testing.assert_array_equal(f64[0].cpu().numpy(), noisy)  # replay is bit-exact
    u8, f32 = ops.denoise_wavelet(f64, "bior1.5", None, out="both")
    f = f32[0].cpu().numpy().astype(np.float64)
    u8 = u8[0].cpu().numpy()
    np.testing.assert_array_equal(got_u8, u8)  # the plugin surface runs exactly these kernels

    err = np.abs(f - ref_f)
    d = u8.astype(int) - ref_u8.astype(int)
    rec = {"var": var, "max_abs_err": float(err.max()), "mean_abs_err": float(err.mean()),
           "u8_flips": int((d != 0).sum()), "u8_flip_share": float((d != 0).mean()),
           "n": int(d.size)}
    print("LIVE_PATH " + json.dumps(rec))
    assert err.max() <= TOL, rec
    check_u8(u8, ref_f, ref_u8)


@pytest.mark.parametrize("wavelet,levels", [("bior1.5", None), ("db1", 3)])
@pytest.mark.parametrize("src", ["u8", "f64"])
def test_wavelet_batch_invariant(dev, wavelet, levels, src):
    """An image's result does not depend on the batch around it: the bior1.5 analysis splits row
    bands by batch size (fewer, longer bands for big batches), but its sums of squares are built
    from per-(thread, 5-row group: WS_G) partials rounded to a power-of-two grid, so every later sum is
    exact and order-free; denoising an image alone and inside a batch of 40 (different row bands
    at every level) gives bit-identical outputs -- a sharded batch equals the 1-GPU run
    (INTEGRATION.md)."""
    import torch
    from idn import ops
    imgs = textured(40, 600, 1000, seed=77)
    x = torch.from_numpy(imgs).cuda()
    if src == "f64":
        x = torch.clamp(x.double() / 255.0 + 0.1 * torch.randn(x.shape, dtype=torch.float64,
                                                               device=x.device,
                                                               generator=torch.Generator(x.device).manual_seed(5)), 0, 1)
    u8_all, f_all = ops.denoise_wavelet(x, wavelet, levels, out="both")
    for i in (0, 17, 39):
        u8_one, f_one = ops.denoise_wavelet(x[i:i + 1], wavelet, levels, out="both")
        assert torch.equal(u8_one[0], u8_all[i]), i
        assert torch.equal(f_one[0], f_all[i]), i
    # and a middle-sized batch (another band count)
    u8_mid, f_mid = ops.denoise_wavelet(x[10:17], wavelet, levels, out="both")
    assert torch.equal(u8_mid, u8_all[10:17])
    assert torch.equal(f_mid, f_all[10:17])


def _plain_keys(x64, wavelet, levels):
    """the colour-range keys the wavelet computes itself (wl_color_minmax) for float64 x64"""
    import torch
    from idn import _lib, ops
    n, h, w, _ = x64.shape
    ops.denoise_wavelet(x64, wavelet, levels, out="u8")
    off = _lib.load().idn_wavelet_stats_offset(n, h, w, ops.WAVELETS[wavelet],
                                               -1 if levels is None else levels)
    ws = ops._WS_CACHE[(str(x64.device), torch.cuda.current_stream(x64.device).cuda_stream)]
    st = ws[off:off + n * 256 * 8].view(torch.int64).view(n, 256)
    return torch.cat([st[:, 200:203], st[:, 203:206]], dim=1).cpu()


@pytest.mark.parametrize("mode,var", [("gaussian", 0.1), ("gaussian", 1.5), ("speckle", 1.0)])
@pytest.mark.parametrize("form", ["offset", "ids", "replay"])
def test_noise_ycc_matches_unfused(dev, mode, var, form):
    """idn_noise_ycc_u8 writes the float64 image random_noise(out='f64') writes (the same draws,
    bit for bit), and its colour-range keys equal the ones the wavelet's own min / max pass
    reduces from that image; the wavelet fed those keys gives the unfused outputs bit for bit"""
    import torch
    from idn import ops
    imgs = textured(3, 600, 1000, seed=19)
    x = torch.from_numpy(imgs).cuda()
    kw = {"var": var, "seed": 7}
    if form == "offset":
        kw["offset"] = 4
    elif form == "ids":
        kw["image_ids"] = [9, 2, 40]
    else:
        rs = np.random.RandomState(3)
        kw["replay"] = torch.from_numpy(rs.normal(0.0, var ** 0.5, imgs.shape)).cuda()
    ref = ops.random_noise(x, mode, out="f64", **kw)
    got, keys = ops.random_noise_ycc(x, mode, **kw)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
    for wavelet, levels in (("bior1.5", None), ("db1", 3)):
        want_keys = _plain_keys(ref, wavelet, levels)
        assert torch.equal(keys.cpu(), want_keys), wavelet
        u8a, fa = ops.denoise_wavelet(ref, wavelet, levels, out="both")
        u8b, fb = ops.denoise_wavelet(got, wavelet, levels, out="both", ycc_keys=keys)
        torch.cuda.synchronize()
        assert torch.equal(u8a, u8b) and torch.equal(fa, fb), wavelet


def test_live_path_uses_the_fused_pair(dev, monkeypatch):
    """Preprocessor on test_v0 'gaussian_wavelet_var*' takes random_noise_ycc -> denoise_wavelet
    with the keys; each image's output equals the two-step composition with its drawn level"""
    import torch
    from idn import ops
    from idn.pipeline import Preprocessor
    x = torch.from_numpy(textured(3, 600, 1000, seed=23)).cuda()
    calls = []
    orig = ops.random_noise_ycc
    monkeypatch.setattr(ops, "random_noise_ycc", lambda *a, **k: calls.append(1) or orig(*a, **k))
    pre = Preprocessor("gaussian_wavelet_var0.1", "test_v0", seed=3, rng=random.Random(5))
    outs, plans = pre(x, image_ids=[0, 1, 2])
    assert calls, "the fused noise kernel did not run"
    for i, (o, p) in enumerate(zip(outs, plans)):
        assert p.steps[0].op == "gaussian" and p.steps[1].op == "wavelet"
        f = ops.random_noise(x[i:i + 1], "gaussian", var=float(p.steps[0].args[0]), seed=3,
                             offset=i, out="f64")
        want = ops.denoise_wavelet(f, p.steps[1].args[0], p.steps[1].args[1])
        assert torch.equal(o, want[0] if want.dim() == 4 else want), i
