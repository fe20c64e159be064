"""GPU: the fused one-pass steps equal the unfused two-step composition bit for bit.

  noise_filter   random_noise (Philox) -> U8 -> cv2.GaussianBlur / cv2.blur
                 (lib/model/test.py:220-241, minibatch.py:115-146; BASELINE config 2)
  gaussian_blob  cv2.GaussianBlur -> prep_im_for_blob (lib/utils/blob.py:33-47)
The unfused steps are themselves pinned to the oracle (test_noise_gpu.py, test_filters_gpu.py,
test_misc_gpu.py), so equality here carries that parity over."""
import numpy as np
import pytest

from conftest import textured

pytestmark = pytest.mark.gpu

SHAPES = [(3, 600, 1000), (2, 37, 40), (1, 9, 336), (2, 130, 1008), (1, 64, 96)]


def _t(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("mode,kw", [("gaussian", {"var": 1.0}), ("speckle", {"var": 0.5}),
                                     ("s&p", {"amount": 0.4})])
@pytest.mark.parametrize("flt,k", [("mean", 3), ("gaus_blur", 3), ("gaus_blur", 5)])
def test_noise_filter_equals_two_steps(dev, shape, mode, kw, flt, k):
    import idn
    x = _t(textured(*shape, seed=sum(shape) + k))
    got = idn.ops.noise_filter(x, mode, flt, k, seed=11, offset=5, form="fused", **kw)
    t = idn.ops.random_noise(x, mode, seed=11, offset=5, out="u8", **kw)
    ref = idn.gaussian_blur(t, k) if flt == "gaus_blur" else idn.blur(t, k)
    assert np.array_equal(got.cpu().numpy(), ref.cpu().numpy())


def test_noise_filter_image_ids(dev):
    import idn
    x = _t(textured(4, 120, 200, seed=2))
    ids = [7, 3, 100, 4]
    got = idn.ops.noise_filter(x, "gaussian", "mean", 3, var=1.0, seed=3, image_ids=ids, form="fused")
    for i, gid in enumerate(ids):
        one = idn.ops.noise_filter(x[i:i + 1], "gaussian", "mean", 3, var=1.0, seed=3, offset=gid, form="fused")
        assert np.array_equal(got[i].cpu().numpy(), one[0].cpu().numpy())


def test_noise_filter_unsupported_layout_falls_back(dev):
    """rows wider than 3024 bytes are not fused: the two-step path gives the same answer."""
    import idn
    x = _t(textured(1, 40, 1100, seed=9))
    got = idn.ops.noise_filter(x, "gaussian", "gaus_blur", 5, var=0.1, seed=1, form="fused")
    ref = idn.gaussian_blur(idn.ops.random_noise(x, "gaussian", var=0.1, seed=1, out="u8"), 5)
    assert np.array_equal(got.cpu().numpy(), ref.cpu().numpy())


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("k", [3, 5])
def test_gaussian_blob_equals_two_steps(dev, shape, k):
    import idn
    x = _t(textured(*shape, seed=sum(shape)))
    got = idn.ops.gaussian_blob(x, k)
    ref = idn.ops.blob(idn.gaussian_blur(x, k))
    assert got.dtype == ref.dtype and np.array_equal(got.cpu().numpy(), ref.cpu().numpy())


@pytest.mark.parametrize("chunk_batch", [1, 5, 70])
def test_noise_filter_pipelined_equals_serial(dev, chunk_batch):
    import idn
    x = _t(textured(chunk_batch, 96, 160, seed=chunk_batch))
    a = idn.ops.noise_filter(x, "gaussian", "mean", 3, var=1.0, seed=2, offset=4, form="serial")
    b = idn.ops.noise_filter(x, "gaussian", "mean", 3, var=1.0, seed=2, offset=4, form="pipelined")
    c = idn.ops.noise_filter(x, "gaussian", "mean", 3, var=1.0, seed=2, offset=4, form="fused")
    import torch
    torch.cuda.synchronize()
    assert np.array_equal(a.cpu().numpy(), b.cpu().numpy())
    assert np.array_equal(a.cpu().numpy(), c.cpu().numpy())
