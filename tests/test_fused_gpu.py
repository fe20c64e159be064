"""GPU: the fused / pipelined steps equal the two-step composition bit for bit.

  noise_filter   random_noise (Philox) -> U8 -> cv2.blur, chunk-pipelined on two streams
                 (lib/model/test.py:220-241, minibatch.py:115-146; BASELINE config 2)
  gaussian_blob  cv2.GaussianBlur -> prep_im_for_blob (lib/utils/blob.py:33-47)
The unfused steps are themselves pinned to the oracle (test_noise_gpu.py, test_filters_gpu.py,
test_misc_gpu.py), so equality here carries that parity over."""
import numpy as np
import pytest

from conftest import textured

pytestmark = pytest.mark.gpu

SHAPES = [(3, 600, 1000), (2, 37, 40), (1, 9, 336), (2, 130, 1008), (1, 64, 96),
          # the pitched tile (rows of 16 k + 8 bytes): band tails, 1-3 segments
          (2, 601, 1000), (1, 19, 344), (2, 7, 680), (1, 6, 24)]


def _t(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("k", [3, 5])
def test_gaussian_blob_equals_two_steps(dev, shape, k):
    import idn
    x = _t(textured(*shape, seed=sum(shape)))
    got = idn.ops.gaussian_blob(x, k)
    ref = idn.ops.blob(idn.gaussian_blur(x, k))
    assert got.dtype == ref.dtype and np.array_equal(got.cpu().numpy(), ref.cpu().numpy())


@pytest.mark.parametrize("knobs", [{"IDN_STENCIL_FORM": "0"}, {"IDN_STENCIL_NTP": "1"},
                                   {"IDN_STENCIL_NTS": "1", "IDN_STENCIL_NTP": "1"}])
def test_gaussian_blob_forms_agree(dev, monkeypatch, knobs):
    """tuning build: the flat tile and the pitched tile's cache policies give the product's blob"""
    import idn
    from idn import _lib
    x = _t(textured(2, 600, 1000, seed=4))
    want = {k: idn.ops.gaussian_blob(x, k).cpu().numpy() for k in (3, 5)}
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    with _lib.variant("tuning"):
        for k in (3, 5):
            assert np.array_equal(idn.ops.gaussian_blob(x, k).cpu().numpy(), want[k]), k


@pytest.mark.parametrize("chunk_batch", [1, 5, 70])
def test_noise_filter_pipelined_equals_serial(dev, chunk_batch):
    import idn
    x = _t(textured(chunk_batch, 96, 160, seed=chunk_batch))
    a = idn.ops.noise_filter(x, "gaussian", "mean", 3, var=1.0, seed=2, offset=4, form="serial")
    b = idn.ops.noise_filter(x, "gaussian", "mean", 3, var=1.0, seed=2, offset=4, form="pipelined")
    import torch
    torch.cuda.synchronize()
    assert np.array_equal(a.cpu().numpy(), b.cpu().numpy())
    t = idn.ops.random_noise(x, "gaussian", var=1.0, seed=2, offset=4, out="u8")
    assert np.array_equal(a.cpu().numpy(), idn.blur(t, 3).cpu().numpy())
