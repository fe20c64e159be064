"""GPU parity of the JPEG decode front-end (cv2.imread, lib/model/test.py:191, minibatch.py:85).

Default mode: bit-exact against the reference's pinned decoder, IJG libjpeg 9d
(requirements.txt:74) -- expected pixels committed in tests/golden/jpeg9.* (full arrays for the
small files, SHA-256 + crops + channel sums for the demo images and the 600x1000 file), made by
tests/golden/make_jpeg9_fixtures.py.  mode="turbo": bit-exact against the GPU box's own Pillow,
which links libjpeg-turbo.  Files: tests/golden/jpeg (the reference's demo images + Pillow-written
cases, progressive files included: the scan path)."""
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"
JPEG = GOLD / "jpeg"
META = json.loads((GOLD / "jpeg9.json").read_text())["files"]
NAMES = sorted(META)


def check_libjpeg9(name, got):
    rec = META[name]
    assert list(got.shape) == rec["shape"], name
    z = np.load(GOLD / "jpeg9.npz")
    if rec.get("full"):
        ref = z[name]
        d = np.abs(got.astype(int) - ref.astype(int))
        assert d.max() == 0, (name, d.max(), np.argwhere(d > 0)[:5])
    else:
        for k, (y, x) in enumerate(rec["crops"]):
            assert np.array_equal(got[y:y + 32, x:x + 32], z[f"{name}:crop{k}"]), (name, k)
        assert [int(got[..., c].astype(np.int64).sum()) for c in range(3)] == rec["sums"], name
    assert hashlib.sha256(np.ascontiguousarray(got).tobytes()).hexdigest() == rec["sha256"], name


def pil_bgr(path):
    """the box Pillow's decode as cv2.imread would return it: BGR; a 4-component file through
    OpenCV's CMYK -> BGR conversion of libjpeg's CMYK output (Pillow reads that inverted)"""
    from PIL import Image
    from oracle import jpeg9
    with Image.open(path) as im:
        if im.mode == "CMYK":
            return jpeg9.cv_cmyk_to_bgr(255 - np.asarray(im).astype(np.int64))
        a = np.asarray(im.convert("RGB"))
    return np.ascontiguousarray(a[..., ::-1])


@pytest.mark.parametrize("name", NAMES)
def test_decode_bitexact_vs_libjpeg9(dev, name):
    from idn import ops
    got = ops.jpeg_decode([(JPEG / name).read_bytes()])[0].cpu().numpy()
    check_libjpeg9(name, got)


@pytest.mark.parametrize("name", NAMES)
def test_decode_turbo_mode_bitexact_vs_pil(dev, name):
    from PIL import features
    if not (features.version("jpg") or "").startswith(("6", "8", "3")):
        pytest.skip("the box's Pillow does not link libjpeg-turbo")
    from idn import ops
    if "smooth" in name:  # libjpeg-turbo's block smoothing is not restated
        from idn._lib import IdnError
        with pytest.raises(IdnError, match="unsupported"):
            ops.jpeg_decode([(JPEG / name).read_bytes()], mode="turbo")
        return
    got = ops.jpeg_decode([(JPEG / name).read_bytes()], mode="turbo")[0].cpu().numpy()
    ref = pil_bgr(JPEG / name)
    d = np.abs(got.astype(int) - ref.astype(int))
    assert d.max() == 0, (name, d.max(), np.argwhere(d > 0)[:5])


def test_batch_of_demo_images_and_imread_gpu(dev):
    from idn import io, ops
    demo = sorted(JPEG.glob("demo_*.jpg"))
    got = ops.jpeg_decode([p.read_bytes() for p in demo]).cpu().numpy()
    for i, p in enumerate(demo):
        check_libjpeg9(p.name, got[i])
    mixed = [JPEG / "s444_q95_96x128.jpg", demo[0], JPEG / "gray_q80_91x77.jpg", demo[1],
             JPEG / "s422_q85_120x200.jpg"]
    outs = io.imread_gpu(mixed)
    for p, o in zip(mixed, outs):
        check_libjpeg9(p.name, o.cpu().numpy())


def test_size_mismatch_and_unsupported_raise(dev):
    from idn import ops
    from idn._lib import IdnError
    with pytest.raises(IdnError, match="size"):
        ops.jpeg_decode([(JPEG / "s444_q95_96x128.jpg").read_bytes(),
                         (JPEG / "s420_q100_64x80.jpg").read_bytes()])
    from test_jpeg import _lossless
    with pytest.raises(IdnError, match="lossless"):
        ops.jpeg_decode([_lossless((JPEG / "s444_q95_96x128.jpg").read_bytes())])
    with pytest.raises(ValueError, match="mode"):
        ops.jpeg_decode([(JPEG / "s444_q95_96x128.jpg").read_bytes()], mode="ijg")


@pytest.mark.parametrize("chunk", [512, 1024])
def test_small_chunks_stress_synchronisation(dev, chunk):
    """512-bit chunks: hundreds of chunks per file, most starting mid-symbol and mid-block; the
    sync passes must still reach the exact trajectory (bit-exact output)"""
    from idn import ops
    for name in NAMES:
        got = ops.jpeg_decode([(JPEG / name).read_bytes()], chunk_bits=chunk)[0].cpu().numpy()
        check_libjpeg9(name, got)


def test_truncated_restart_file_decodes_without_fault(dev):
    """a DRI file that lost its tail (fewer RST markers than intervals): the missing intervals
    start at the end of the data instead of at uninitialised offsets (libjpeg only warns)"""
    from idn import ops
    data = (JPEG / "s420_rstrow_120x160.jpg").read_bytes()
    sos = data.index(b"\xff\xda")
    cut = sos + (len(data) - sos) // 2
    trunc = data[:cut] + b"\xff\xd9"
    good = ops.jpeg_decode([data])[0].cpu().numpy()
    got = ops.jpeg_decode([trunc])[0].cpu().numpy()
    assert got.shape == good.shape
    # the intervals before the cut decode exactly as in the whole file
    assert np.array_equal(got[:16], good[:16])


def test_smoothed_and_plain_files_in_one_batch(dev):
    """block smoothing is per image (JpegDev.smooth and its coef_bits latch): one launch of
    96x128 files -- baseline, complete progressive, two smoothed ones (Al 1 luma / Cb; never-coded
    chroma AC) and the DC-less cut that libjpeg leaves unsmoothed -- each as libjpeg 9d decodes it"""
    from idn import ops
    names = ["prog_smooth_cut_s444_96x128.jpg", "s444_q95_96x128.jpg",
             "prog_smooth_dconly_s444_96x128.jpg", "prog_s444_q85_96x128.jpg",
             "prog_nodc_cut_s444_96x128.jpg", "prog_smooth_cut_s444_96x128.jpg"]
    got = ops.jpeg_decode([(JPEG / n).read_bytes() for n in names]).cpu().numpy()
    for i, n in enumerate(names):
        check_libjpeg9(n, got[i])


def test_mixed_baseline_and_progressive_batch(dev):
    """one launch holding baseline files (the parallel path) and progressive ones (the scan path)
    of the same size: every image as its own decode"""
    from idn import ops
    names = ["s420_q90_600x1000.jpg", "prog_s420_q90_600x1000.jpg", "s420_q90_600x1000.jpg",
             "prog_s420_q90_600x1000.jpg"]
    got = ops.jpeg_decode([(JPEG / n).read_bytes() for n in names]).cpu().numpy()
    for i, n in enumerate(names):
        check_libjpeg9(n, got[i])
    small = ["prog_s444_q85_96x128.jpg", "s444_q95_96x128.jpg"]
    got = ops.jpeg_decode([(JPEG / n).read_bytes() for n in small]).cpu().numpy()
    for i, n in enumerate(small):
        check_libjpeg9(n, got[i])


def test_truncated_progressive_file_decodes_without_fault(dev):
    """a progressive file cut inside its last scan (libjpeg's script: the luma AC refinement,
    restart markers every 4 blocks): every scan header is there (no smoothing case), the data runs
    out -- the decoder reads zeros past it (libjpeg's fill).  The restart intervals complete before
    the cut decode exactly as in the whole file, so every pixel row whose luma blocks all lie in
    those intervals equals the whole file's decode; the rows after the cut differ"""
    from idn import ops
    from test_jpeg import _sos_offsets
    data = (JPEG / "prog_s420_rst4_120x160.jpg").read_bytes()
    last = _sos_offsets(data)[-1]
    ns = data[last + 4]
    assert ns == 1 and data[last + 5] == 1  # one component, the luma (component id 1)
    hdr_end = last + 2 + ((data[last + 2] << 8) | data[last + 3])
    cut = last + (len(data) - last) // 2
    trunc = data[:cut] + b"\xff\xd9"
    k = data.find(b"\xff\xdd")  # DRI: restart interval in MCUs (= blocks in this scan)
    assert k > 0 and k < last
    dri = (data[k + 4] << 8) | data[k + 5]
    seg = data[hdr_end:cut]
    nrst = sum(1 for i in range(len(seg) - 1) if seg[i] == 0xFF and 0xD0 <= seg[i + 1] <= 0xD7)
    wib = (160 + 7) // 8  # luma blocks per row
    rows_ok = 8 * ((nrst * dri) // wib)  # pixel rows whose luma blocks all precede the cut
    assert 8 <= rows_ok < 120
    good = ops.jpeg_decode([data])[0].cpu().numpy()
    got = ops.jpeg_decode([trunc])[0].cpu().numpy()
    assert got.shape == good.shape
    assert np.array_equal(got[:rows_ok], good[:rows_ok])
    assert not np.array_equal(got[rows_ok + 8:], good[rows_ok + 8:])


def test_large_mixed_batch_bitexact_and_errors(dev):
    """a 96-file batch of baseline and progressive files in mixed order (the gather runs in parts
    of the batch, each copied as soon as it is complete): every image as its own decode, in
    order, and an unsupported file late in the batch still fails the whole call"""
    from idn import ops
    from idn._lib import IdnError
    names = ["s420_q90_600x1000.jpg", "prog_s420_q90_600x1000.jpg"]
    datas = [(JPEG / n).read_bytes() for n in names]
    order = [(i * 7 + i // 5) % 2 for i in range(96)]
    got = ops.jpeg_decode([datas[k] for k in order]).cpu().numpy()
    first = {k: got[order.index(k)] for k in (0, 1)}
    for k in (0, 1):
        check_libjpeg9(names[k], first[k])
    for i, k in enumerate(order):
        assert np.array_equal(got[i], first[k]), i
    from test_jpeg import _lossless
    bad = [datas[0]] * 96
    bad[90] = _lossless(datas[0])
    with pytest.raises(IdnError, match="unsupported|lossless"):
        ops.jpeg_decode(bad)


# ---- damaged files: libjpeg's treatment of bad data (tests/golden/jpeg_damage.py) ---------------
def _damaged():
    import sys
    if str(GOLD) not in sys.path:
        sys.path.insert(0, str(GOLD))
    import jpeg_damage
    return jpeg_damage


DAMAGED = json.loads((GOLD / "jpeg9_damaged.json").read_text())["cases"]


def check_damaged(key, got):
    rec = DAMAGED[key]
    assert list(got.shape) == rec["shape"], key
    if hashlib.sha256(np.ascontiguousarray(got).tobytes()).hexdigest() != rec["sha256"]:
        rows = np.load(GOLD / "jpeg9_damaged.npz")[key]
        bad = np.nonzero((got.astype(np.int64).sum(axis=1) != rows).any(axis=1))[0]
        raise AssertionError(f"{key}: rows differ from {bad[:1]} ({len(bad)} rows)")


@pytest.mark.parametrize("case", _damaged().cases(), ids=lambda c: _damaged().key(c))
def test_damaged_file_matches_libjpeg9(dev, case):
    """cut files, bit errors, bad Huffman codes, lost / renumbered restart markers and stray markers
    decode as the real libjpeg 9d decodes them (cv2.imread returns the image, with warnings):
    every decoder -- the chunked one, restart intervals, the scan path, arithmetic"""
    from idn import ops
    jd = _damaged()
    data = jd.damage((JPEG / case[0]).read_bytes(), case[1], case[2])
    check_damaged(jd.key(case), ops.jpeg_decode([data])[0].cpu().numpy())


def test_damaged_files_small_chunks_and_one_batch(dev):
    """the chunked decoder's end-of-data rule with 512-bit chunks (many chunks past the end of a cut
    file), and every damaged variant of a file in one batch with the intact file"""
    from idn import ops
    jd = _damaged()
    for name in ["s444_q95_96x128.jpg", "gray_q80_91x77.jpg", "s420_opt_130x170.jpg"]:
        cs = [c for c in jd.cases() if c[0] == name]
        src = (JPEG / name).read_bytes()
        datas = [jd.damage(src, c[1], c[2]) for c in cs]
        for c, d in zip(cs, datas):
            check_damaged(jd.key(c), ops.jpeg_decode([d], chunk_bits=512)[0].cpu().numpy())
        got = ops.jpeg_decode([src] + datas).cpu().numpy()
        check_libjpeg9(name, got[0])
        for k, c in enumerate(cs):
            check_damaged(jd.key(c), got[k + 1])


def test_damaged_files_turbo_mode_match_the_oracle(dev):
    """mode="turbo" on damaged baseline / arithmetic files against the oracle's turbo mode (pinned
    by tests/test_jpeg.py against libjpeg-turbo's C code)"""
    from idn import ops
    from oracle import jpeg9
    jd = _damaged()
    for c in jd.cases():
        if "600x1000" in c[0] or not c[0].startswith(("s4", "gray", "arith_s", "arith_rst")):
            continue
        data = jd.damage((JPEG / c[0]).read_bytes(), c[1], c[2])
        got = ops.jpeg_decode([data], mode="turbo")[0].cpu().numpy()
        assert np.array_equal(got, jpeg9.imread(data, mode="turbo")), jd.key(c)


@pytest.mark.parametrize("chunk", [0, 512, 4096])
def test_restart_intervals_decode_as_the_same_image_without_them(dev, chunk):
    """restart intervals go through the chunked decoder, each interval cut into its own chunks:
    a 600x1000 image written with a restart marker every MCU row (38 long intervals), every 3
    MCUs (short ones) and without any has the same coefficients, so the same pixels, in a mixed
    batch and at any chunk size"""
    import io
    from PIL import Image
    from idn import ops
    rng = np.random.default_rng(5)
    y, x = np.mgrid[0:600, 0:1000]
    img = np.stack([(x * 0.3 + 50 * np.sin(y / 13.0)) % 256, (y * 0.5) % 256, (x + y) % 256], -1)
    img = np.clip(img + rng.normal(0, 10, img.shape), 0, 255).astype(np.uint8)
    files = []
    for kw in ({}, {"restart_marker_rows": 1}, {"restart_marker_blocks": 3}):
        b = io.BytesIO()
        Image.fromarray(img).save(b, "JPEG", quality=90, subsampling=2, **kw)
        files.append(b.getvalue())
    assert files[1].count(b"\xff\xdd") == 1 and files[2].count(b"\xff\xdd") == 1
    got = ops.jpeg_decode(files + files[::-1], chunk_bits=chunk).cpu().numpy()
    for k in range(1, 6):
        assert np.array_equal(got[k], got[0]), k
    check = ops.jpeg_decode([files[1]], mode="turbo", chunk_bits=chunk)[0].cpu().numpy()
    assert np.array_equal(check, ops.jpeg_decode([files[0]], mode="turbo")[0].cpu().numpy())


def test_random_damaged_files_match_the_oracle(dev):
    """150 random damages (tests/golden/jpeg_damage.py random_damage: cuts, bit flips, one-bit runs,
    stray markers, renumbered restart markers) of the small fixtures, GPU against the oracle (itself
    pinned to libjpeg 9d by the committed damaged variants); tools/jpeg_fuzz.py runs more"""
    import random
    from idn import ops
    from idn._lib import IdnError
    from oracle import jpeg9
    jdm = _damaged()
    rng = random.Random(11)
    files = [p for p in sorted(JPEG.glob("*.jpg")) if p.stat().st_size < 20000]
    for i in range(150):
        p = rng.choice(files)
        data = jdm.random_damage(p.read_bytes(), rng)
        try:
            ref = jpeg9.imread(data)
        except Exception:
            with pytest.raises(IdnError):
                ops.jpeg_decode([data])
            continue
        got = ops.jpeg_decode([data])[0].cpu().numpy()
        assert np.array_equal(got, ref), (i, p.name)


# ---- cv2.imread's EXIF orientation (OpenCV 3.4.2 loadsave.cpp ApplyExifOrientation) -------------
EXIF = GOLD / "jpeg_exif"
EXIF_META = json.loads((GOLD / "jpeg_exif.json").read_text())["files"]


def check_exif(name, got):
    rec = EXIF_META[name]
    assert list(got.shape) == rec["shape"], name
    z = np.load(GOLD / "jpeg_exif.npz")
    if rec.get("full"):
        d = np.abs(got.astype(int) - z[name].astype(int))
        assert d.max() == 0, (name, d.max(), np.argwhere(d > 0)[:5])
    else:
        for k, (y, x) in enumerate(rec["crops"]):
            assert np.array_equal(got[y:y + 32, x:x + 32], z[f"{name}:crop{k}"]), (name, k)
    assert hashlib.sha256(np.ascontiguousarray(got).tobytes()).hexdigest() == rec["sha256"], name


@pytest.mark.parametrize("name", sorted(EXIF_META))
def test_exif_orientation_bitexact(dev, name):
    """each of the eight orientations (baseline 4:2:0, progressive 4:2:2, grayscale, restart rows,
    600x1000) and the malformed EXIF blocks: the real libjpeg 9d decode turned as OpenCV 3.4.2
    turns it (tests/golden/make_jpeg_exif.py)"""
    from idn import ops
    got = ops.jpeg_decode([(EXIF / name).read_bytes()])[0].cpu().numpy()
    check_exif(name, got)


def test_exif_orientations_in_one_batch_and_ignore_flag(dev):
    """the transposed orientations 5..8 of one file share a launch with an unturned file of the
    transposed size; IMREAD_IGNORE_ORIENTATION returns every one as decoded; imread_gpu groups by
    the turned size"""
    from idn import io, ops
    from oracle import jpeg9
    names = [f"s420_o{o}_37x53.jpg" for o in (5, 6, 7, 8)] + [f"prog_s422_o{o}_45x67.jpg" for o in (6, 8)]
    datas = [(EXIF / n).read_bytes() for n in names[:4]]
    got = ops.jpeg_decode(datas).cpu().numpy()
    for n, g in zip(names, got):
        check_exif(n, g)
    plain = ops.jpeg_decode(datas, orientation=False).cpu().numpy()
    base = jpeg9.decode(datas[0])
    for g in plain:
        assert np.array_equal(g, base)
    paths = [EXIF / n for n in names] + [EXIF / "s420_o1_37x53.jpg", EXIF / "s420_o3_37x53.jpg"]
    outs = io.imread_gpu(paths)
    for p, o in zip(paths, outs):
        check_exif(p.name, o.cpu().numpy())
    outs = io.imread_gpu(paths, orientation=False)
    assert [tuple(o.shape) for o in outs[:4]] == [(37, 53, 3)] * 4
    from idn._lib import IdnError
    with pytest.raises(IdnError, match="size"):  # 53x37 turned against 37x53 unturned
        ops.jpeg_decode([datas[0], (EXIF / "s420_o1_37x53.jpg").read_bytes()])


def test_exif_turbo_mode_turns_too(dev):
    """the turn is OpenCV's step after the library's decode: the turbo mode applies it as well"""
    from idn import ops
    from oracle import exif
    for name in ("s420_o6_37x53.jpg", "prog_s422_o7_45x67.jpg", "gray_o3_29x41.jpg"):
        data = (EXIF / name).read_bytes()
        got = ops.jpeg_decode([data], mode="turbo")[0].cpu().numpy()
        ref = exif.apply(pil_bgr(EXIF / name), EXIF_META[name]["orientation"])
        assert np.array_equal(got, ref), name


def test_image_reader_prefetch_matches_imread_gpu(dev):
    """idn.io.ImageReader (the test loop's reads, test.py:189-191, decoded in windows with the
    next window decoded ahead on a side stream): every image equals imread_gpu's, in order and on demand out of
    order, and the per-image body run on its images (noise + wavelet + blob, the bench's
    detect_e2e_pipelined) gives the same blobs as on imread_gpu's"""
    import torch
    from idn import detect_blob
    from idn import io as idn_io
    names = sorted(p.name for p in JPEG.glob("demo_*.jpg"))
    assert len(names) >= 3
    paths = [str(JPEG / n) for n in names] * 2
    ref = [idn_io.imread_gpu([p])[0] for p in paths]
    for batch in (1, 4, 8):  # windows of mixed sizes (several decode launches) and a partial one
        with idn_io.ImageReader(paths, batch=batch) as rd:
            for i in range(len(paths)):
                assert torch.equal(rd[i], ref[i]), (batch, paths[i])
            assert torch.equal(rd[1], ref[1])  # out of order: its window decoded on demand
    import random
    with idn_io.ImageReader(paths) as rd:
        for i in range(len(paths)):
            random.seed(1000 + i)  # test_v0 draws the gaussian level from the random module
            a = detect_blob.apply_noise(rd[i], "gaussian_wavelet_var0.1", mode="test_v0",
                                        image_id=i, as_tensor=True)
            random.seed(1000 + i)
            b = detect_blob.apply_noise(ref[i], "gaussian_wavelet_var0.1", mode="test_v0",
                                        image_id=i, as_tensor=True)
            ba, _ = detect_blob._get_blobs(a)
            bb, _ = detect_blob._get_blobs(b)
            np.testing.assert_array_equal(ba["data"], bb["data"])
