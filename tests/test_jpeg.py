"""CPU tests of the JPEG decode front-end's host side: the marker parser
through the C-ABI (no GPU needed), on the fixture files of tests/golden/make_jpeg_fixtures.py."""
from pathlib import Path

import pytest

JPEG = Path(__file__).resolve().parent / "golden" / "jpeg"


def _files():
    return sorted(p for p in JPEG.glob("*.jpg") if not p.name.startswith("progressive"))


def test_info_matches_pil():
    from PIL import Image
    from idn import ops
    assert len(_files()) >= 16
    for p in _files():
        with Image.open(p) as im:
            w, h = im.size
            c = 1 if im.mode == "L" else 3
        assert ops.jpeg_info(p.read_bytes()) == (h, w, c), p.name


def test_unsupported_and_corrupt_raise():
    from idn import ops
    from idn._lib import IdnError
    with pytest.raises(IdnError, match="progressive"):
        ops.jpeg_info((JPEG / "progressive_64x64.jpg").read_bytes())
    with pytest.raises(IdnError, match="SOI"):
        ops.jpeg_info(b"not a jpeg at all")
    data = (JPEG / "s444_q95_96x128.jpg").read_bytes()
    with pytest.raises(IdnError):
        ops.jpeg_info(data[:40])  # truncated inside the headers


def test_workspace_size():
    import ctypes
    from idn import _lib, ops
    lib = _lib.load()
    datas = [p.read_bytes() for p in _files()[:3]]
    bufs, ptrs, lens = ops._file_ptrs(datas)
    assert lib.idn_jpeg_workspace_size(ptrs, lens, 3) > sum(lens)
    bufs, ptrs, lens = ops._file_ptrs([(JPEG / "progressive_64x64.jpg").read_bytes()])
    assert lib.idn_jpeg_workspace_size(ptrs, lens, 1) == 0
    del ctypes
