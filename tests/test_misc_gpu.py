"""GPU parity: float64 stencils, shader, bloom, float64 blob, INTER_LINEAR resize and the drop-in
blob builders (lib/utils/blob.py, lib/model/test.py:_get_blobs) vs the oracle."""
import random

import numpy as np
import pytest

from conftest import textured

pytestmark = pytest.mark.gpu


def _t(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _np(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


def _f64_img(shape, seed):
    rs = np.random.RandomState(seed)
    img = textured(*shape, seed=seed)
    return np.clip(img * (1.0 / 255.0) + rs.normal(0, 0.3, img.shape), 0, 1)


F64_SHAPES = [(2, 37, 53), (1, 600, 1000), (1, 2, 5), (1, 1, 7)]


@pytest.mark.parametrize("shape", F64_SHAPES)
@pytest.mark.parametrize("k", [3, 5])
def test_gaussian_blur_f64_bitexact(dev, shape, k):
    import idn
    import oracle
    x = _f64_img(shape, sum(shape) + k)
    got = _np(idn.ops.gaussian_blur_f64(_t(x), k))
    ref = oracle.cvf.gaussian_blur_f64(x, k)
    assert np.array_equal(got, ref), np.abs(got - ref).max()


@pytest.mark.parametrize("shape", F64_SHAPES)
def test_blur_f64(dev, shape):
    """cv2.blur's 64F path uses running sums; the direct sum agrees to a few ulp (tol 1e-13)."""
    import idn
    import oracle
    x = _f64_img(shape, sum(shape))
    got = _np(idn.ops.blur_f64(_t(x), 3))
    ref = oracle.cvf.blur_f64(x, 3)
    assert np.abs(got - ref).max() <= 1e-13


@pytest.mark.parametrize("factor", [3.0, 0.5, 1.7, 1.0])
def test_shader_bitexact(dev, factor):
    import idn
    import oracle
    img = textured(2, 45, 67, seed=int(factor * 10))
    got = _np(idn.ops.shader(_t(img), factor))
    ref = np.stack([oracle.automold.shader(im, factor) for im in img])
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("shape", [(2, 375, 500), (1, 600, 1000), (1, 300, 64)])
def test_bloom_vs_sequential_oracle(dev, shape):
    """48 circle+addWeighted passes evaluated per pixel vs the literal sequential version."""
    import idn
    import oracle
    img = textured(*shape, seed=sum(shape))
    got = _np(idn.ops.bloom(_t(img), rng=random.Random(11)))
    rng = random.Random(11)
    ref = np.stack([oracle.automold.add_sun_flare(im, rng) for im in img])
    d = np.abs(got.astype(int) - ref.astype(int))
    assert d.max() <= 1 and (d > 0).mean() < 1e-4, (d.max(), (d > 0).mean())


def test_bloom_rejects_short_images(dev):
    """rng.randint(1, h // 100 - 2) raises for h < 300, as in the reference."""
    import idn
    with pytest.raises(ValueError):
        idn.ops.bloom(_t(textured(1, 120, 80)), rng=random.Random(1))


@pytest.mark.parametrize("flip", [False, True])
def test_blob_from_f64_bitexact(dev, flip):
    import idn
    x = _f64_img((2, 41, 59), 7) * 255.0
    got = _np(idn.ops.blob_from_f64(_t(x), flip=flip))
    ref = []
    for im in x:
        if flip:
            im = im[:, ::-1]
        f = im.astype(np.float32, copy=True)
        f -= np.array([[[102.9801, 115.9465, 122.7717]]])
        ref.append(f)
    assert np.array_equal(got, np.stack(ref))


@pytest.mark.parametrize("hw,scale", [((375, 500), 1.6), ((600, 1000), 1.0), ((333, 500), 1.8018),
                                      ((480, 640), 1.25), ((64, 96), 0.5), ((37, 53), 2.7),
                                      ((1000, 600), 0.6)])
def test_resize_linear_bitexact(dev, hw, scale):
    import idn
    import oracle
    rs = np.random.RandomState(hw[0])
    x = (rs.uniform(-128, 128, size=(*hw, 3))).astype(np.float32)
    got = _np(idn.ops.resize_linear(_t(x), scale, scale))
    ref = oracle.cvf.resize_linear_f32(x, scale, scale)
    assert got.shape == ref.shape
    assert np.array_equal(got, ref), np.abs(got - ref).max()


def test_prep_im_for_blob_and_list(dev):
    """blob.py:33-47 + 17-30 on u8 and float64 inputs of different sizes (zero padding)."""
    from idn import blobs as blob
    import oracle
    ims = [textured(1, 375, 500, seed=1)[0], _f64_img((1, 333, 500), 2)[0] * 255.0]
    got_ims, scales = [], []
    for im in ims:
        f, s = blob.prep_im_for_blob(im, np.array([[[102.9801, 115.9465, 122.7717]]]), 600, 1000)
        got_ims.append(f)
        scales.append(s)
    got = blob.im_list_to_blob(got_ims)
    ref_ims = []
    for im in ims:
        f = im.astype(np.float32, copy=True)
        f -= np.array([[[102.9801, 115.9465, 122.7717]]])
        s = blob.im_scale_for(f.shape, 600, 1000)
        ref_ims.append(oracle.cvf.resize_linear_f32(f, s, s))
    assert scales == [1.6, 600 / 333]
    hmax = max(r.shape[0] for r in ref_ims)
    wmax = max(r.shape[1] for r in ref_ims)
    assert got.shape == (2, hmax, wmax, 3)
    for i, r in enumerate(ref_ims):
        assert np.array_equal(got[i, :r.shape[0], :r.shape[1]], r)
        assert not got[i, r.shape[0]:].any() and not got[i, :, r.shape[1]:].any()


def test_get_blobs_test_path(dev):
    from idn import detect_blob
    import oracle
    im = textured(1, 480, 640, seed=9)[0]
    blobs, scales = detect_blob._get_blobs(im)
    f = im.astype(np.float32, copy=True)
    f -= np.array([[[102.9801, 115.9465, 122.7717]]])
    ref = oracle.cvf.resize_linear_f32(f, 1.25, 1.25)
    assert scales.tolist() == [1.25]
    assert np.array_equal(blobs["data"][0], ref)
