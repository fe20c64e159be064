"""CPU tests of the JPEG decode front-end (cv2.imread at lib/model/test.py:191,
lib/roi_data_layer/minibatch.py:85).

* the oracle (oracle/jpeg9.py, a restatement of IJG libjpeg 9d's sequential and progressive
  decode) against the
  real libjpeg 9d decode of every fixture (tests/golden/jpeg9.*, made by
  tests/golden/make_jpeg9_fixtures.py from conda Pillow 8.4.0 linked with libjpeg.so.9), and its
  libjpeg-turbo mode against this container's Pillow (turbo);
* the host side of the HIP library through the C-ABI (marker parser, table validation, workspace
  sizing; no GPU needed)."""
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

GOLD = Path(__file__).resolve().parent / "golden"
JPEG = GOLD / "jpeg"


def _files():
    return sorted(JPEG.glob("*.jpg"))


def _lossless(data: bytes) -> bytes:
    """the same file relabelled lossless (SOF0 -> SOF3): a format the decoder rejects"""
    k = data.index(b"\xff\xc0")
    return data[:k + 1] + b"\xc3" + data[k + 2:]


def _sos_offsets(data: bytes):
    out, k = [], data.find(b"\xff\xda")
    while k >= 0:
        out.append(k)
        k = data.find(b"\xff\xda", k + 2)
    return out


def _meta():
    return json.loads((GOLD / "jpeg9.json").read_text())


def test_fixture_set_is_complete():
    meta = _meta()
    assert meta["libjpeg"].startswith("9")
    assert sorted(meta["files"]) == [p.name for p in _files()]
    assert len(meta["files"]) >= 24
    assert sum(n.startswith("prog") for n in meta["files"]) >= 6


@pytest.mark.parametrize("name", [p.name for p in _files()
                                  if p.stat().st_size < 20000 or p.name.startswith("demo_0004")])
def test_oracle_libjpeg9_matches_real_libjpeg9(name):
    from oracle import jpeg9
    rec = _meta()["files"][name]
    got = jpeg9.imread((JPEG / name).read_bytes())
    assert list(got.shape) == rec["shape"]
    if rec.get("full"):
        ref = np.load(GOLD / "jpeg9.npz")[name]
        d = np.abs(got.astype(int) - ref.astype(int))
        assert d.max() == 0, (name, d.max(), np.argwhere(d > 0)[:5])
    assert hashlib.sha256(got.tobytes()).hexdigest() == rec["sha256"]


@pytest.mark.parametrize("name", ["s420_q100_64x80.jpg", "s422_q85_120x200.jpg",
                                  "s444_q95_96x128.jpg", "s420_q75_odd_37x53.jpg",
                                  "progressive_64x64.jpg", "prog_s422_q75_odd_45x67.jpg",
                                  "prog_s420_rst4_120x160.jpg", "prog_gray_q80_91x77.jpg"] +
                         [p.name for p in _files() if p.name.startswith("cs_")] +
                         [p.name for p in _files() if p.name.startswith("arith_") and
                          "smooth" not in p.name] +
                         [p.name for p in _files() if p.name.startswith(("cmyk", "ycck"))])
def test_oracle_turbo_mode_matches_system_pil(name):
    from PIL import Image
    from oracle import jpeg9
    with Image.open(JPEG / name) as im:
        if im.mode == "CMYK":  # libjpeg's CMYK output (Pillow reads it inverted) through OpenCV's
            ref = jpeg9.cv_cmyk_to_bgr(255 - np.asarray(im).astype(np.int64))
        else:
            ref = np.asarray(im.convert("RGB"))[..., ::-1]
    assert np.array_equal(jpeg9.imread((JPEG / name).read_bytes(), mode="turbo"), ref)


def test_libjpeg9_and_turbo_differ_on_subsampled_files():
    """the reason for the re-pin: the two libraries disagree on every 4:2:x file"""
    from oracle import jpeg9
    data = (JPEG / "s420_q75_odd_37x53.jpg").read_bytes()
    assert not np.array_equal(jpeg9.imread(data), jpeg9.imread(data, mode="turbo"))


def test_info_matches_pil():
    from PIL import Image
    from idn import ops
    for p in _files():
        with Image.open(p) as im:
            w, h = im.size
            c = {"L": 1, "CMYK": 4}.get(im.mode, 3)
        assert ops.jpeg_info(p.read_bytes()) == (h, w, c), p.name


def test_unsupported_and_corrupt_raise():
    from idn import ops
    from idn._lib import IdnError
    assert ops.jpeg_info((JPEG / "progressive_64x64.jpg").read_bytes()) == (64, 64, 3)
    with pytest.raises(IdnError, match="lossless"):
        ops.jpeg_info(_lossless((JPEG / "s444_q95_96x128.jpg").read_bytes()))
    with pytest.raises(IdnError, match="SOI"):
        ops.jpeg_info(b"not a jpeg at all")
    data = (JPEG / "s444_q95_96x128.jpg").read_bytes()
    with pytest.raises(IdnError):
        ops.jpeg_info(data[:40])  # truncated inside the headers


def _ws(datas, flags=0):
    from idn import _lib, ops
    bufs, ptrs, lens = ops._file_ptrs(datas)
    return _lib.load().idn_jpeg_workspace_size(ptrs, lens, len(datas), flags)


def test_workspace_size():
    datas = [p.read_bytes() for p in _files()[:3]]
    assert _ws(datas) > sum(map(len, datas))
    assert _ws([_lossless((JPEG / "s444_q95_96x128.jpg").read_bytes())]) == 0
    assert _ws([(JPEG / "progressive_64x64.jpg").read_bytes()]) > 0
    # libjpeg 9's full-size chroma planes need more room than turbo's subsampled ones
    d = [(JPEG / "s420_q90_600x1000.jpg").read_bytes()]
    assert _ws(d, 0) > _ws(d, 1) > 0
    assert _ws(d, 1 | (512 << 8)) > 0
    assert _ws(d, 4) == 0 and _ws(d, 100 << 8) == 0  # unknown flag bit, chunk < 512


def _dht_segments(data):
    i, out = 2, []
    while i + 4 <= len(data):
        m, ln = data[i + 1], (data[i + 2] << 8) | data[i + 3]
        if m == 0xC4:
            out.append(i + 4)
        if m == 0xDA:
            break
        i += 2 + ln
    return out


def test_malformed_huffman_table_is_rejected_before_use():
    """jdhuff.c: a code length whose codes do not fit (or end all ones) is JERR_BAD_HUFF_TABLE.
    Counts moved to length 1 keep the segment's size valid, so only the table check catches it
    (before the fix the fast-lookup fill ran past its 512 entries)."""
    data = bytearray((JPEG / "s444_q95_96x128.jpg").read_bytes())
    k = _dht_segments(data)[0]
    bits = data[k + 1:k + 17]
    total = sum(bits)
    assert total >= 3
    new = [3] + [0] * 15
    rest = total - 3
    for ln in range(15, 0, -1):  # put the rest at the longest length, keeping the sum
        if rest:
            new[ln] = rest
            rest = 0
    data[k + 1:k + 17] = bytes(new)
    assert _ws([bytes(data)]) == 0
    from idn import ops
    assert ops.jpeg_info(bytes(data))[0] == 96  # headers still parse


def test_sos_length_checked_before_reading():
    data = (JPEG / "s444_q95_96x128.jpg").read_bytes()
    k = data.index(b"\xff\xda")
    from idn import ops
    from idn._lib import IdnError
    with pytest.raises(IdnError):
        ops.jpeg_info(data[:k] + b"\xff\xda\x00\x02")


def test_imread_lossless_formats_through_pil(tmp_path):
    """io.imread without OpenCV: non-JPEG (lossless) files are PIL-decoded and flipped to BGR;
    no GPU is touched (JPEGs go to the GPU decoder: tests/test_minibatch_gpu.py)"""
    import importlib.util
    from PIL import Image
    from idn import io
    if importlib.util.find_spec("cv2") is not None:
        pytest.skip("OpenCV present: io.imread is cv2.imread itself")
    rgb = np.random.RandomState(0).randint(0, 256, (9, 13, 3)).astype(np.uint8)
    Image.fromarray(rgb).save(tmp_path / "a.png")
    assert np.array_equal(io.imread(tmp_path / "a.png"), rgb[..., ::-1])
    # 16-bit grayscale: OpenCV's png_set_strip_16 keeps the high byte (PIL's convert would clip);
    # palette and gray + alpha: expanded / alpha dropped.  (cv2 is absent here: the OpenCV
    # behaviour is restated from grfmt_png.cpp, parity-unpinned)
    g16 = np.random.RandomState(1).randint(0, 65536, (7, 11)).astype(np.uint16)
    Image.fromarray(g16, "I;16").save(tmp_path / "g16.png")
    assert np.array_equal(io.imread(tmp_path / "g16.png"),
                          np.repeat((g16 >> 8).astype(np.uint8)[..., None], 3, -1))
    pal = Image.fromarray(rgb).quantize(16)
    pal.save(tmp_path / "p.png")
    assert np.array_equal(io.imread(tmp_path / "p.png"), np.asarray(pal.convert("RGB"))[..., ::-1])
    la = np.stack([rgb[..., 0], rgb[..., 1]], -1)
    Image.fromarray(la, "LA").save(tmp_path / "la.png")
    assert np.array_equal(io.imread(tmp_path / "la.png"), np.repeat(la[..., :1], 3, -1))
    with pytest.raises(FileNotFoundError):
        io.imread(tmp_path / "missing.png")


def test_progressive_scan_script_of_the_fixtures():
    """the progressive fixtures carry libjpeg's standard script: DC first / refine and AC first /
    refine scans, i.e. all four progressive decoders are exercised"""
    kinds = set()
    for p in _files():
        if not p.name.startswith("prog"):
            continue
        data = p.read_bytes()
        for k in _sos_offsets(data):
            ns = data[k + 4]
            ss, se, ahal = data[k + 5 + 2 * ns:k + 8 + 2 * ns]
            kinds.add(("DC" if ss == 0 else "AC") + ("_refine" if ahal >> 4 else "_first"))
    assert kinds == {"DC_first", "DC_refine", "AC_first", "AC_refine"}


def test_progressive_without_final_scans_is_smoothed():
    """a progressive file whose last scans are missing leaves AC coefficients imprecise; libjpeg
    9d block-smooths it (jdcoefct.c smoothing_ok / decompress_smooth_data).  The fixtures
    prog_smooth_*.jpg cover it (Al > 0 caps, never-coded chroma AC, grayscale, odd 4:2:2, restart
    intervals) and test_oracle_libjpeg9_matches_real_libjpeg9 pins the oracle's smoothing to the
    real library; here: the host parser takes them, the smoothing changes pixels (so those tests
    are not vacuous), and libjpeg-turbo mode refuses them (turbo smooths differently)"""
    from idn import ops
    from oracle import jpeg9
    names = [p.name for p in _files() if p.name.startswith("prog_smooth")]
    assert len(names) >= 5
    gold = np.load(GOLD / "jpeg9.npz")
    for name in names:
        data = (JPEG / name).read_bytes()
        d = jpeg9.parse_and_decode(data)
        assert d["smooth"] is not None, name
        assert ops.jpeg_info(data)[0] == d["height"]
        unsmoothed = dict(d, smooth=None)
        orig = jpeg9.parse_and_decode
        try:
            jpeg9.parse_and_decode = lambda _b: unsmoothed
            plain = jpeg9.imread(data)
        finally:
            jpeg9.parse_and_decode = orig
        assert (plain != gold[name]).mean() > 0.05, name
        with pytest.raises(NotImplementedError):
            jpeg9.imread(data, mode="turbo")


def test_progressive_smoothing_ok_mirrors_libjpeg():
    """libjpeg 9d smooths a progressive file only if EVERY component has DC data and nonzero
    Q00 Q01 Q10 Q20 Q11 Q02 (jdcoefct.c smoothing_ok): a file with imprecise AC but no DC scans,
    or with a zero chroma Q01, decodes unsmoothed -- accepted by the host parser and the oracle,
    whose pixels test_oracle_libjpeg9_matches_real_libjpeg9 pins to the real library"""
    from idn import ops
    from oracle import jpeg9
    for name in ("prog_nodc_cut_s444_96x128.jpg", "prog_q0_cut_s444_96x128.jpg"):
        data = (JPEG / name).read_bytes()
        assert ops.jpeg_info(data) == (96, 128, 3), name
        assert jpeg9.imread(data).shape == (96, 128, 3)


# (libjpeg 9d, libjpeg-turbo) colour space of each derived colour-space fixture
# (tests/golden/make_jpeg_fixtures.py colorspaces(); observed with conda Pillow 8.4 / libjpeg 9 and
# the system Pillow / libjpeg-turbo when the fixtures were made)
_CS = {"cs_rgbids_jfif_s444_96x128.jpg": ("rgb", "ycc"),
       "cs_rgbids_s420_odd_37x53.jpg": ("rgb", "rgb"),
       "cs_adobe0_s444_96x128.jpg": ("ycc", "rgb"),
       "cs_adobe0_ids012_prog_s422_45x67.jpg": ("rgb", "rgb"),
       "cs_adobe1_rgbids_s422_120x200.jpg": ("rgb", "ycc")}


def test_colour_space_rules_of_both_libraries():
    """jdapimin.c default_decompress_parms: libjpeg 9 decides RGB / YCbCr by the component IDs
    first, libjpeg-turbo by the JFIF / Adobe markers first; the five fixtures separate the two
    orders (their pixels are pinned by test_oracle_libjpeg9_matches_real_libjpeg9 and
    test_oracle_turbo_mode_matches_system_pil)"""
    from oracle import jpeg9
    assert sorted(_CS) == sorted(p.name for p in _files() if p.name.startswith("cs_"))
    for name, (nine, turbo) in _CS.items():
        d = jpeg9.parse_and_decode((JPEG / name).read_bytes())
        assert (jpeg9.color_space(d, "libjpeg9"), jpeg9.color_space(d, "turbo")) == (nine, turbo)


def test_extension_markers_and_big_gamut_are_rejected():
    """JPGn / DHP / EXP markers stop libjpeg-turbo (and JPG8 is libjpeg 9's LSE colour transform),
    big-gamut component IDs select a colour space that is not restated: IdnError, not a decode"""
    from idn import ops
    from idn._lib import IdnError
    from oracle import jpeg9
    data = (JPEG / "s444_q95_96x128.jpg").read_bytes()
    lse = data[:2] + b"\xff\xf8\x00\x04\x0d\x00" + data[2:]
    with pytest.raises(IdnError, match="extension marker"):
        ops.jpeg_info(lse)
    with pytest.raises(ValueError):
        jpeg9.imread(lse)
    k = data.find(b"\xff\xc0")
    bg = bytearray(data)
    for c, v in enumerate((0x72, 0x67, 0x62)):  # 'r' 'g' 'b' (scan selectors left: IDs only)
        bg[k + 10 + 3 * c] = v
    with pytest.raises(ValueError):
        jpeg9.imread(bytes(bg))


def test_arithmetic_fixtures_cover_the_coder():
    """arithmetic-coded fixtures (jpegtran -arithmetic of libjpeg 9, tests/golden/make_jpeg_fixtures.py
    arithmetic()): SOF9 sequential and SOF10 progressive, restart intervals, 4:4:4 / 4:2:2 /
    4:2:0 / grayscale, and a cut progressive file that is block-smoothed.  Their pixels are pinned
    by test_oracle_libjpeg9_matches_real_libjpeg9; the host parser takes them"""
    from idn import ops
    from oracle import jpeg9
    names = [p.name for p in _files() if p.name.startswith("arith_")]
    sofs, rst, smooth = set(), False, False
    for name in names:
        data = (JPEG / name).read_bytes()
        sofs |= {m for m in (0xC9, 0xCA) if bytes([0xFF, m]) in data[:data.find(b"\xff\xda")]}
        rst |= b"\xff\xdd" in data
        smooth |= jpeg9.parse_and_decode(data)["smooth"] is not None
        assert ops.jpeg_info(data)[2] in (1, 3)
    assert len(names) >= 7 and sofs == {0xC9, 0xCA} and rst and smooth


def test_four_component_files():
    """CMYK (Adobe transform 0, or no Adobe marker) and YCCK (transform 2) files, baseline and
    progressive: libjpeg 9d's CMYK output (ycck_cmyk_convert for YCCK) pinned by the real library
    (tests/golden/jpeg9.*), then OpenCV's CMYK -> BGR (restated, parity-unpinned: cv2 is not
    importable here)"""
    from idn import ops
    from oracle import jpeg9
    names = [p.name for p in _files() if p.name.startswith(("cmyk", "ycck"))]
    assert len(names) >= 4
    spaces = set()
    for name in names:
        data = (JPEG / name).read_bytes()
        assert ops.jpeg_info(data)[2] == 4
        spaces.add(jpeg9.color_space(jpeg9.parse_and_decode(data), "libjpeg9"))
    assert spaces == {"cmyk", "ycck"}


# ---- damaged files (tests/golden/jpeg_damage.py): what libjpeg does where the data is bad ----------
def _damaged():
    import sys
    if str(GOLD) not in sys.path:
        sys.path.insert(0, str(GOLD))
    import jpeg_damage
    return jpeg_damage


def _damaged_meta():
    return json.loads((GOLD / "jpeg9_damaged.json").read_text())


def _damaged_cases(big: bool):
    """the 600x1000 file's cases take the pure-Python oracle a minute each: only the cut early"""
    out = []
    for c in _damaged().cases():
        if "600x1000" in c[0] and not (big or (c[1] == "cut" and c[2] <= 0.3)):
            continue
        out.append(c)
    return out


def test_damaged_fixture_set_is_complete():
    jd = _damaged()
    meta = _damaged_meta()
    assert meta["libjpeg"].startswith("9")
    assert sorted(meta["cases"]) == sorted(jd.key(c) for c in jd.cases())
    ops = {c[1] for c in jd.cases()}
    assert ops == {"cut", "cutrst", "flip", "ones", "junk", "rstnum", "shortiv"}
    for c in jd.cases():  # every recipe changes the file (a cut at 0.97 may keep all the data)
        data = (JPEG / c[0]).read_bytes()
        assert jd.damage(data, c[1], c[2]) != data or c[1] == "cut", c


@pytest.mark.parametrize("case", _damaged_cases(False), ids=lambda c: _damaged().key(c))
def test_oracle_matches_libjpeg9_on_damaged_files(case):
    """jdhuff.c / jdarith.c / jdmarker.c on bad data, restated (oracle/jpeg9.py _entropy,
    _intervals, _Bits): an MCU is decoded only while its interval's data lasted up to its start,
    past the data the bits are 0, a bit pattern that is no code takes 17 bits and decodes as 0,
    and at every restart the marker is taken or resynchronised by jpeg_resync_to_restart's three
    actions -- pinned against the real libjpeg 9d's pixels"""
    from oracle import jpeg9
    jd = _damaged()
    rec = _damaged_meta()["cases"][jd.key(case)]
    got = jpeg9.imread(jd.damage((JPEG / case[0]).read_bytes(), case[1], case[2]))
    assert list(got.shape) == rec["shape"]
    if hashlib.sha256(got.tobytes()).hexdigest() != rec["sha256"]:
        rows = np.load(GOLD / "jpeg9_damaged.npz")[jd.key(case)]
        bad = np.nonzero((got.astype(np.int64).sum(axis=1) != rows).any(axis=1))[0]
        raise AssertionError(f"{jd.key(case)}: rows differ from {bad[:1]} ({len(bad)} rows)")


_TURBO_DAMAGED = ("s4", "gray", "arith_s", "arith_rst")


def test_oracle_turbo_mode_matches_system_pil_on_damaged_files(tmp_path):
    """libjpeg-turbo's entropy decoders treat bad data as libjpeg 9d's do: the system Pillow's
    decode of the damaged baseline and arithmetic files.  Its SIMD IDCT saturates differently on
    the out-of-range coefficients damaged data can give, so Pillow runs here with libjpeg-turbo's C
    code (JSIMD_FORCENONE, read once per process: a child process)"""
    import os
    import subprocess
    import sys
    jd = _damaged()
    cases = [c for c in _damaged_cases(False) if "600x1000" not in c[0] and
             c[0].startswith(_TURBO_DAMAGED)]
    assert len(cases) >= 90
    out = tmp_path / "pil.npz"
    script = (
        "import io, sys, numpy as np\n"
        "from pathlib import Path\n"
        "from PIL import Image\n"
        f"sys.path.insert(0, {str(GOLD)!r})\n"
        "import jpeg_damage as jd\n"
        "res = {}\n"
        "for c in jd.cases():\n"
        "    if '600x1000' in c[0] or not c[0].startswith(%r): continue\n"
        f"    d = jd.damage(Path({str(JPEG)!r}, c[0]).read_bytes(), c[1], c[2])\n"
        "    with Image.open(io.BytesIO(d)) as im:\n"
        "        res[jd.key(c)] = np.asarray(im.convert('RGB'))[..., ::-1]\n"
        f"np.savez({str(out)!r}, **res)\n") % (_TURBO_DAMAGED,)
    subprocess.run([sys.executable, "-c", script], check=True,
                   env=dict(os.environ, JSIMD_FORCENONE="1"))
    from oracle import jpeg9
    ref = np.load(out)
    for c in cases:
        data = jd.damage((JPEG / c[0]).read_bytes(), c[1], c[2])
        assert np.array_equal(jpeg9.imread(data, mode="turbo"), ref[jd.key(c)]), jd.key(c)


# ---- cv2.imread's EXIF orientation (OpenCV 3.4.2 loadsave.cpp ApplyExifOrientation) -------------
EXIF = GOLD / "jpeg_exif"


def _exif_meta():
    return json.loads((GOLD / "jpeg_exif.json").read_text())["files"]


def test_exif_fixture_set():
    meta = _exif_meta()
    assert sorted(meta) == sorted(p.name for p in EXIF.glob("*.jpg"))
    assert {r["orientation"] for r in meta.values()} == set(range(1, 9))
    # the malformed cases: OpenCV's reader gives up where Pillow's still finds a tag
    assert sum(r["orientation"] == 1 and r["pil_orientation"] not in (None, 1)
               for r in meta.values()) >= 6


@pytest.mark.parametrize("name", sorted(_exif_meta()) if (GOLD / "jpeg_exif.json").exists() else [])
def test_exif_orientation_oracle_and_library(name):
    """oracle/exif.py and the library's idn_jpeg_orientation (host code, no GPU) give the
    orientation recorded for the fixture; on well-formed Pillow-written blocks that is Pillow's
    own reading of the tag"""
    from oracle import exif
    from idn import ops
    rec = _exif_meta()[name]
    data = (EXIF / name).read_bytes()
    assert exif.orientation(data) == rec["orientation"]
    assert ops.jpeg_orientation(data) == rec["orientation"]
    if "_o" in name and not any(k in name for k in ("bad", "trunc", "xmp", "dup", "o0", "o9",
                                                    "len6", "mark")):
        assert rec["pil_orientation"] == rec["orientation"]
    h, w, c = rec["shape"]
    assert ops.jpeg_info(data)[:2] == (h, w)
    if rec["orientation"] >= 5:
        assert ops.jpeg_info(data, orientation=False)[:2] == (w, h)


@pytest.mark.parametrize("name", [n for n in sorted(_exif_meta()) if "600x1000" not in n]
                         if (GOLD / "jpeg_exif.json").exists() else [])
def test_exif_oracle_imread_matches_libjpeg9_turned_by_pillow(name):
    """the oracle's imread (libjpeg 9d restatement + the EXIF step) against the real libjpeg 9d
    decode turned by Pillow's Image.transpose (an independent statement of the eight turns)"""
    from oracle import jpeg9
    rec = _exif_meta()[name]
    got = jpeg9.imread((EXIF / name).read_bytes())
    assert np.array_equal(got, np.load(GOLD / "jpeg_exif.npz")[name])
    assert hashlib.sha256(got.tobytes()).hexdigest() == rec["sha256"]


def test_exif_orientation_fuzz_library_vs_oracle():
    """random damage to EXIF blocks (bytes of the TIFF header, IFD counts, offsets, tag types and
    values; cut APP1 lengths; files cut inside the block): the library's host parser and the
    oracle agree on every file"""
    from oracle import exif
    from idn import ops
    rs = np.random.RandomState(7)
    seeds = [(EXIF / n).read_bytes() for n in sorted(_exif_meta()) if "600x1000" not in n]
    for k in range(1500):
        data = bytearray(seeds[rs.randint(len(seeds))])
        k1 = data.find(b"\xff\xe1")
        if k1 < 0:
            continue
        end = k1 + 4 + 64
        for _ in range(rs.randint(1, 4)):
            j = rs.randint(k1 + 2, min(end, len(data)))
            data[j] = rs.randint(256) if rs.rand() < 0.7 else data[j] ^ (1 << rs.randint(8))
        if rs.rand() < 0.1:
            data = data[:rs.randint(2, k1 + 60)]
        data = bytes(data)
        assert ops.jpeg_orientation(data) == exif.orientation(data), (k, data[:k1 + 80].hex())
