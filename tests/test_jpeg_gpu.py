"""GPU parity of the JPEG decode front-end (cv2.imread, lib/model/test.py:191,
minibatch.py:85) against PIL's decode of the same files (libjpeg-turbo defaults: ISLOW IDCT,
fancy upsampling, integer YCbCr tables -- what cv2.imread also uses), converted to BGR.
Bit-exact.  Files: tests/golden/jpeg (the reference's demo images + Pillow-written cases)."""
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
JPEG = Path(__file__).resolve().parent / "golden" / "jpeg"


def pil_bgr(path):
    from PIL import Image
    with Image.open(path) as im:
        a = np.asarray(im.convert("RGB"))
    return np.ascontiguousarray(a[..., ::-1])


@pytest.mark.parametrize("name", sorted(p.name for p in JPEG.glob("*.jpg")
                                        if not p.name.startswith("progressive")))
def test_decode_bitexact_vs_pil(dev, name):
    from idn import ops
    got = ops.jpeg_decode([(JPEG / name).read_bytes()])[0].cpu().numpy()
    ref = pil_bgr(JPEG / name)
    assert got.shape == ref.shape
    d = np.abs(got.astype(int) - ref.astype(int))
    assert d.max() == 0, (name, d.max(), np.argwhere(d > 0)[:5])


def test_batch_of_demo_images_and_imread_gpu(dev):
    from idn import io, ops
    demo = sorted(JPEG.glob("demo_*.jpg"))
    got = ops.jpeg_decode([p.read_bytes() for p in demo]).cpu().numpy()
    for i, p in enumerate(demo):
        assert np.array_equal(got[i], pil_bgr(p)), p.name
    mixed = [JPEG / "s444_q95_96x128.jpg", demo[0], JPEG / "gray_q80_91x77.jpg", demo[1]]
    outs = io.imread_gpu(mixed)
    for p, o in zip(mixed, outs):
        assert np.array_equal(o.cpu().numpy(), pil_bgr(p)), p.name


def test_size_mismatch_and_unsupported_raise(dev):
    from idn import ops
    from idn._lib import IdnError
    with pytest.raises(IdnError, match="size"):
        ops.jpeg_decode([(JPEG / "s444_q95_96x128.jpg").read_bytes(),
                         (JPEG / "s420_q100_64x80.jpg").read_bytes()])
    with pytest.raises(IdnError):
        ops.jpeg_decode([(JPEG / "progressive_64x64.jpg").read_bytes()])


@pytest.mark.parametrize("chunk", ["512", "1024"])
def test_small_chunks_stress_synchronisation(dev, monkeypatch, chunk):
    """512-bit chunks: hundreds of chunks per file, most starting mid-symbol and mid-block; the
    sync passes must still reach the exact trajectory (bit-exact output)"""
    from idn import ops
    monkeypatch.setenv("IDN_JPEG_CHUNK", chunk)
    for p in sorted(JPEG.glob("*.jpg")):
        if p.name.startswith("progressive"):
            continue
        got = ops.jpeg_decode([p.read_bytes()])[0].cpu().numpy()
        assert np.array_equal(got, pil_bgr(p)), (chunk, p.name)
