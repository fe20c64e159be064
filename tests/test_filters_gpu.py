"""GPU parity: HIP stencil / median / bilateral filters vs the C oracle (oracle/filters.c).

Integer filters must be bit-exact.  Shapes cover the fast path's segment tails (row bytes
% 16 == 0 and == 8), multi-segment rows, the 600x1000 BASELINE shape, tiny images (vertical
reflection of h < ksize) and shapes only the generic path accepts (W*C % 8 != 0).
"""
import ctypes

import numpy as np
import pytest

from conftest import textured

pytestmark = pytest.mark.gpu

SHAPES = [
    (2, 600, 1000),  # BASELINE shape: 3 segments of 1000 B, tail 8
    (3, 64, 96),     # rb 288: one segment, tail 8
    (2, 40, 104),    # rb 312: tail 0
    (1, 33, 336),    # rb 1008: exactly one full segment
    (2, 17, 344),    # rb 1032: two segments
    (1, 5, 16),      # rb 48, h 5
    (2, 2, 24),      # h 2 < ksize
    (1, 1, 40),      # single row
    (2, 37, 53),     # rb 159: generic path
    (1, 9, 11),      # generic path, tiny
]


def _run(fn, img, *args):
    import torch
    x = torch.from_numpy(img).cuda()
    y = fn(x, *args)
    torch.cuda.synchronize()
    return y.cpu().numpy()


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("k", [3, 5])
def test_gaussian_blur_bitexact(dev, shape, k):
    import idn
    import oracle
    img = textured(*shape, seed=sum(shape) + k)
    got = _run(idn.gaussian_blur, img, k)
    ref = oracle.cv.gaussian_blur(img, k)
    assert np.array_equal(got, ref), f"mismatches: {np.argwhere(got != ref)[:8]}"


@pytest.mark.parametrize("shape", SHAPES)
def test_box_blur_bitexact(dev, shape):
    import idn
    import oracle
    img = textured(*shape, seed=sum(shape))
    got = _run(idn.blur, img, 3)
    ref = oracle.cv.blur(img, 3)
    assert np.array_equal(got, ref), f"mismatches: {np.argwhere(got != ref)[:8]}"


@pytest.mark.parametrize("k", [3, 5])
def test_stencil_random_extremes(dev, k):
    """i.i.d. full-range bytes incl. all-0 / all-255 rows exercise the SWAR lane bounds."""
    import idn
    import oracle
    rs = np.random.RandomState(k)
    img = rs.randint(0, 256, size=(2, 50, 1000, 3)).astype(np.uint8)
    img[0, :7] = 255
    img[1, -6:] = 0
    img[1, :, :5] = 255
    for fn, ref in ((idn.gaussian_blur, oracle.cv.gaussian_blur(img, k)),):
        assert np.array_equal(_run(fn, img, k), ref)
    if k == 3:
        assert np.array_equal(_run(idn.blur, img, 3), oracle.cv.blur(img, 3))


@pytest.mark.parametrize("shape", SHAPES[:8] + [(3, 600, 1000)])
@pytest.mark.parametrize("form", ["0"])
def test_stencil_tile_fetch_forms(dev, monkeypatch, shape, form):
    """IDN_STENCIL_GLDS=0 (tuning build): the register-staged tile fetch (the product fetches the
    tile by global_load_lds_dwordx4) -- bit-exact with the oracle like the product form"""
    import idn
    import oracle
    from idn import _lib
    monkeypatch.setenv("IDN_STENCIL_GLDS", form)
    img = textured(*shape, seed=sum(shape) + 7)
    with _lib.variant("tuning"):
        for k in (3, 5):
            assert np.array_equal(_run(idn.gaussian_blur, img, k), oracle.cv.gaussian_blur(img, k))
        assert np.array_equal(_run(idn.blur, img, 3), oracle.cv.blur(img, 3))


# rows of 16 k + 8 bytes take the pitched tile (round 5): one, two and three segments (a 24-byte
# last segment at rb 2040), band tails (h % 6), the first / last band's reflected rows
PITCHED = [(1, 5, 24), (2, 6, 104), (1, 7, 344), (2, 13, 664), (1, 29, 680), (2, 600, 1000),
           (1, 601, 1000), (1, 3, 1000), (3, 64, 40)]


@pytest.mark.parametrize("shape", PITCHED)
def test_stencil_pitched_tile(dev, shape):
    """the pitched LDS tile (rows of 16 k + 8 bytes) against the oracle for all three filters"""
    import idn
    import oracle
    img = textured(*shape, seed=sum(shape) + 11)
    for k in (3, 5):
        got = _run(idn.gaussian_blur, img, k)
        ref = oracle.cv.gaussian_blur(img, k)
        assert np.array_equal(got, ref), (k, np.argwhere(got != ref)[:8])
    got = _run(idn.blur, img, 3)
    ref = oracle.cv.blur(img, 3)
    assert np.array_equal(got, ref), np.argwhere(got != ref)[:8]


@pytest.mark.parametrize("knobs", [{"IDN_STENCIL_FORM": "0"}, {"IDN_STENCIL_NTP": "1"},
                                   {"IDN_STENCIL_NTP": "2", "IDN_STENCIL_NTS": "1"},
                                   {"IDN_STENCIL_NTS": "1"}, {"IDN_STENCIL_NTP": "1", "IDN_STENCIL_SAUX": "16"},
                                   {"IDN_STENCIL_NTP": "0", "IDN_STENCIL_NTS": "0"}])
@pytest.mark.parametrize("shape", [(2, 600, 1000), (1, 13, 664), (2, 7, 104)])
def test_stencil_forms_and_policies_agree(dev, monkeypatch, knobs, shape):
    """tuning build: the flat tile (IDN_STENCIL_FORM=0) and the pitched tile's cache policies
    (nontemporal private rows / every row, nontemporal stores) give the product's bytes"""
    import idn
    from idn import _lib
    img = textured(*shape, seed=sum(shape) + 5)
    want = {k: _run(idn.gaussian_blur, img, k) for k in (3, 5)}
    want_box = _run(idn.blur, img, 3)
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    with _lib.variant("tuning"):
        for k in (3, 5):
            assert np.array_equal(_run(idn.gaussian_blur, img, k), want[k]), k
        assert np.array_equal(_run(idn.blur, img, 3), want_box)


def test_gaussian_headline_batch(dev):
    """the bench's own launch: 256 x 600 x 1000 x 3 in one call (76,800 workgroup items).  Three
    images (first, middle, last) bit-exact against the oracle, and the whole batch equal to 256
    one-image launches of the same images"""
    import torch
    import idn
    import oracle
    n = 256
    base = torch.from_numpy(textured(1, 600, 1000, seed=21)).cuda()
    # distinct images: the textured base shifted and noised per image on the device
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    x = torch.empty((n, 600, 1000, 3), dtype=torch.uint8, device="cuda")
    for i in range(0, n, 32):
        m = min(32, n - i)
        noise = torch.randint(0, 256, (m, 600, 1000, 3), generator=g, device="cuda",
                              dtype=torch.uint8)
        x[i:i + m] = torch.where(noise < 16, noise, base.expand(m, -1, -1, -1).roll(i, 2))
    y = idn.gaussian_blur(x, 5)
    torch.cuda.synchronize()
    for i in (0, n // 2, n - 1):
        img = x[i:i + 1].cpu().numpy()
        assert np.array_equal(y[i:i + 1].cpu().numpy(), oracle.cv.gaussian_blur(img, 5)), i
    per = torch.empty_like(y)
    for i in range(n):
        idn.gaussian_blur(x[i:i + 1], 5, out=per[i:i + 1])
    torch.cuda.synchronize()
    assert torch.equal(per, y)


def test_generic_path_forced(dev, monkeypatch):
    """the per-pixel kernel (shapes the lane layout does not take), forced on a shape it would
    not get by itself through the tools-only tuning build"""
    import idn
    import oracle
    from idn import _lib
    monkeypatch.setenv("IDN_FORCE_GENERIC", "1")
    img = textured(2, 31, 200, seed=9)
    with _lib.variant("tuning"):
        assert np.array_equal(_run(idn.gaussian_blur, img, 5), oracle.cv.gaussian_blur(img, 5))
        assert np.array_equal(_run(idn.blur, img, 3), oracle.cv.blur(img, 3))
    # and without forcing: c = 2 and odd row lengths take it in the product library
    img2 = textured(2, 17, 45, c=2, seed=4)
    assert np.array_equal(_run(idn.gaussian_blur, img2, 5), oracle.cv.gaussian_blur(img2, 5))


def _run_strided(fn_name, img, k, pad=8):
    """the C-ABI on rows padded to W*C + pad bytes (the stripe form from HBM)"""
    import torch
    from idn import _lib
    lib = _lib.load()
    n, h, w, c = img.shape
    rs = (w * c + pad + 7) // 8 * 8
    buf = torch.zeros((n, h, rs), dtype=torch.uint8, device="cuda")
    buf[:, :, : w * c] = torch.from_numpy(img.reshape(n, h, w * c)).cuda()
    out = torch.full_like(buf, 77)
    rc = getattr(lib, fn_name)(buf.data_ptr(), out.data_ptr(), n, h, w, c, rs, k, None)
    assert rc == 0
    torch.cuda.synchronize()
    assert bool((out[:, :, w * c:] == 77).all())  # padding untouched
    return out[:, :, : w * c].cpu().numpy().reshape(n, h, w, c)


@pytest.mark.parametrize("layout", ["compact", "strided"])
@pytest.mark.parametrize("shape", [(2, 100, 1000), (1, 37, 336), (2, 13, 104), (1, 601, 1000),
                                   (1, 26, 1000), (1, 25, 664)])
def test_stencil_forms_agree(dev, layout, shape):
    """both memory forms of the stencil (the LDS band tile for compact rows, the stripe form for
    strided rows) give cv2's bytes (band tails, 1-3 segments, odd heights)"""
    import idn
    import oracle
    img = textured(*shape, seed=sum(shape))
    for k in (3, 5):
        got = (_run(idn.gaussian_blur, img, k) if layout == "compact"
               else _run_strided("idn_gaussian_blur_u8", img, k))
        assert np.array_equal(got, oracle.cv.gaussian_blur(img, k)), k
    got = _run(idn.blur, img, 3) if layout == "compact" else _run_strided("idn_box_blur_u8", img, 3)
    assert np.array_equal(got, oracle.cv.blur(img, 3))


@pytest.mark.parametrize("w,pad", [(1000, 8), (344, 16), (1400, 0)])
def test_stencil_row_stride_and_wide_rows(dev, w, pad):
    """row_stride > W*C (strided rows take the stripe form) and rows wider than the LDS tile"""
    import torch
    import idn
    import oracle
    from idn import _lib
    lib = _lib.load()
    img = textured(2, 41, w, seed=w + pad)
    wp = w + pad // 3 if pad else w
    rs = wp * 3 + (pad % 3) if pad else w * 3
    rs = (rs + 7) // 8 * 8
    buf = torch.zeros((2, 41, rs), dtype=torch.uint8, device="cuda")
    buf[:, :, : w * 3] = torch.from_numpy(img.reshape(2, 41, w * 3)).cuda()
    out = torch.full_like(buf, 77)
    for k in (3, 5):
        rc = lib.idn_gaussian_blur_u8(buf.data_ptr(), out.data_ptr(), 2, 41, w, 3, rs, k, None)
        assert rc == 0
        torch.cuda.synchronize()
        got = out[:, :, : w * 3].cpu().numpy().reshape(2, 41, w, 3)
        assert np.array_equal(got, oracle.cv.gaussian_blur(img, k)), k
        assert bool((out[:, :, w * 3:] == 77).all())  # padding untouched


def test_rejects_cpu_tensor():
    import torch
    import idn
    with pytest.raises(ValueError):
        idn.gaussian_blur(torch.zeros(4, 4, 3, dtype=torch.uint8), 5)


# + the 5x5 median's 24-byte-lane path (rows of 24k bytes, 1512-byte segments): one exactly full
# segment, a 24-byte second segment, four segments
MEDIAN_SHAPES = SHAPES + [(1, 9, 504), (1, 11, 512), (1, 20, 1600)]


@pytest.mark.parametrize("shape", MEDIAN_SHAPES)
@pytest.mark.parametrize("k", [3, 5])
def test_median_blur_bitexact(dev, shape, k):
    import idn
    import oracle
    img = textured(*shape, seed=sum(shape) * 7 + k)
    got = _run(idn.median_blur, img, k)
    ref = oracle.cv.median_blur(img, k)
    assert np.array_equal(got, ref), f"mismatches: {np.argwhere(got != ref)[:8]}"


@pytest.mark.parametrize("k", [3, 5])
def test_median_saltpepper_extremes(dev, k):
    """s&p-like data (config 3): runs of 0 / 255 around real values, incl. all-equal windows"""
    import idn
    import oracle
    rs = np.random.RandomState(40 + k)
    img = textured(2, 60, 1000, seed=k)
    m = rs.random_sample(img.shape)
    img[m < 0.2] = 0
    img[(m >= 0.2) & (m < 0.4)] = 255
    img[0, 10:20] = 255
    assert np.array_equal(_run(idn.median_blur, img, k), oracle.cv.median_blur(img, k))


def test_median_generic_forced(dev, monkeypatch):
    import idn
    import oracle
    from idn import _lib
    monkeypatch.setenv("IDN_FORCE_GENERIC", "1")
    img = textured(2, 23, 64, seed=5)
    with _lib.variant("tuning"):
        for k in (3, 5):
            assert np.array_equal(_run(idn.median_blur, img, k), oracle.cv.median_blur(img, k))


BILATERAL_CASES = [(9, 20.0, 100.0), (9, 75.0, 75.0), (5, 30.0, 10.0), (3, 10.0, 10.0)]


@pytest.mark.parametrize("shape", [(2, 64, 96), (1, 37, 53), (1, 600, 1000), (2, 5, 7), (1, 9, 1),
                                   (2, 7, 2), (1, 70, 65)])
@pytest.mark.parametrize("case", BILATERAL_CASES)
def test_bilateral_within_1lsb(dev, shape, case):
    """<= 1 LSB vs OpenCV semantics (fp32 sum order / exp ulps); pre-round values within 1e-4 rel"""
    import idn
    import oracle
    d, sc, ss = case
    img = textured(*shape, seed=d + int(sc))
    got = _run(idn.bilateral_filter, img, d, sc, ss)
    ref = oracle.cv.bilateral_filter(img, d, sc, ss)
    diff = np.abs(got.astype(np.int32) - ref.astype(np.int32))
    assert diff.max() <= 1
    # any 1-LSB difference must sit on a rounding boundary of the exact value
    pre = oracle.cv.bilateral_prefilter_f32(img, d, sc, ss)
    frac = np.abs(pre - np.floor(pre) - 0.5)
    assert np.all(frac[diff > 0] < 1e-3)
    assert (diff > 0).mean() < 1e-3


@pytest.mark.parametrize("shape", [(2, 64, 300), (1, 37, 53), (1, 600, 1000), (2, 7, 2)])
@pytest.mark.parametrize("case", BILATERAL_CASES)
def test_bilateral_shared_weights_bitwise(dev, monkeypatch, shape, case):
    """the two-column kernel's shared own-output weights and constant centre weight (product)
    against looking every tap up (IDN_BL2_SYM=0, tuning build): each output's fp32 sum keeps its
    order, so the bytes are identical"""
    import idn
    from idn import _lib
    d, sc, ss = case
    img = textured(*shape, seed=d + 7)
    got = _run(idn.bilateral_filter, img, d, sc, ss)
    monkeypatch.setenv("IDN_BL2_SYM", "0")
    with _lib.variant("tuning"):
        ref = _run(idn.bilateral_filter, img, d, sc, ss)
    np.testing.assert_array_equal(got, ref)


def test_bilateral_recip_exact(dev):
    """the two-column kernel's 1 / wsum (v_rcp_f32 + one Newton step) equals the IEEE quotient
    for every float in [1, 128), the range of its weight sums"""
    import torch
    from idn import _lib
    lib = _lib.load()
    bad = lib.idn_internal_bl_recip_check(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert bad == 0


def test_bilateral_gray(dev):
    import idn
    import oracle
    img = textured(1, 40, 64, c=1, seed=3)
    got = _run(idn.bilateral_filter, img, 9, 20.0, 100.0)
    ref = oracle.cv.bilateral_filter(img, 9, 20.0, 100.0)
    assert np.abs(got.astype(int) - ref.astype(int)).max() <= 1


@pytest.mark.parametrize("form", [{}, {"IDN_MEDIAN_MAP": "0", "IDN_MEDIAN_ROWS": "32"},
                                  {"IDN_MEDIAN_MAP": "1", "IDN_MEDIAN_ROWS": "16"},
                                  {"IDN_MEDIAN_MAP": "2", "IDN_MEDIAN_ROWS": "7"},
                                  {"IDN_MEDIAN_W24": "0", "IDN_MEDIAN_ROWS": "32"},
                                  {"IDN_MEDIAN_PAIR": "0", "IDN_MEDIAN_ROWS": "9"},
                                  {"IDN_MEDIAN_ROWS": "5"}],
                         ids=lambda f: "-".join(f"{k[11:]}{v}" for k, v in f.items()) or "product")
@pytest.mark.parametrize("shape", [(2, 100, 1000), (1, 37, 336), (1, 601, 1000), (2, 13, 104)])
def test_median_forms_agree(dev, monkeypatch, form, shape):
    """every band / workgroup mapping of the median (the tuning build's knobs; {} = the product
    library) gives cv2's bytes (band tails, 1-3 segments)"""
    import contextlib
    import idn
    import oracle
    from idn import _lib
    for k, v in form.items():
        monkeypatch.setenv(k, v)
    img = textured(*shape, seed=sum(shape) + 1)
    with (_lib.variant("tuning") if form else contextlib.nullcontext()):
        for k in (3, 5):
            assert np.array_equal(_run(idn.median_blur, img, k), oracle.cv.median_blur(img, k)), k
