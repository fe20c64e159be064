"""Fixtures for the GPU JPEG decode front-end (tests/test_jpeg*.py).

* the reference's own sample images, copied as data: /root/reference/data/demo/*.jpg (VOC, 500x375,
  baseline 4:2:0) -> tests/golden/jpeg/demo_*.jpg
* synthetic files written by Pillow 12.2 (libjpeg-turbo 3.x encoder) covering what the decoder
  takes: 4:2:0 / 4:2:2 / 4:4:4, grayscale, restart intervals (per row and every 3 MCUs), odd sizes,
  quality 10 .. 100, optimised Huffman tables, and progressive files (SOF2) of every sampling,
  grayscale, odd sizes and restart intervals.

Expected pixels: the reference's pinned IJG libjpeg 9d decode, committed as data by
tests/golden/make_jpeg9_fixtures.py (run under /opt/conda/bin/python3.9); the libjpeg-turbo mode
is compared with the GPU box's own Pillow (turbo) at test time.

  python tests/golden/make_jpeg_fixtures.py
"""
import io
import shutil
from pathlib import Path

import numpy as np
from PIL import Image

OUT = Path(__file__).resolve().parent / "jpeg"
DEMO = Path("/root/reference/data/demo")


def textured(h, w, seed):
    rs = np.random.RandomState(seed)
    y, x = np.mgrid[0:h, 0:w]
    base = 128 + 60 * np.sin(x / 17.0 + seed) * np.cos(y / 23.0) + rs.normal(0, 18, (h, w))
    img = np.stack([base, np.roll(base, 7, 1) * 0.8 + 30, 255 - base], -1)
    return np.clip(img, 0, 255).astype(np.uint8)


def save(name, arr, **kw):
    b = io.BytesIO()
    Image.fromarray(arr).save(b, "JPEG", **kw)
    (OUT / name).write_bytes(b.getvalue())


def main():
    OUT.mkdir(exist_ok=True)
    if DEMO.is_dir():
        for f in sorted(DEMO.glob("*.jpg")):
            shutil.copyfile(f, OUT / f"demo_{f.name}")
    save("s420_q90_600x1000.jpg", textured(600, 1000, 1), quality=90, subsampling=2)
    save("s420_q75_odd_37x53.jpg", textured(37, 53, 2), quality=75, subsampling=2)
    save("s422_q85_120x200.jpg", textured(120, 200, 3), quality=85, subsampling=1)
    save("s444_q95_96x128.jpg", textured(96, 128, 4), quality=95, subsampling=0)
    save("s420_q100_64x80.jpg", textured(64, 80, 5), quality=100, subsampling=2)
    save("s420_q10_75x99.jpg", textured(75, 99, 6), quality=10, subsampling=2)
    save("s420_opt_130x170.jpg", textured(130, 170, 7), quality=80, subsampling=2, optimize=True)
    save("s420_rstrow_120x160.jpg", textured(120, 160, 8), quality=80, subsampling=2,
         restart_marker_rows=1)
    save("s444_rst3_70x90.jpg", textured(70, 90, 9), quality=85, subsampling=0,
         restart_marker_blocks=3)
    save("gray_q80_91x77.jpg", textured(91, 77, 10)[..., 0], quality=80)
    save("gray_rst2_48x64.jpg", textured(48, 64, 11)[..., 0], quality=70, restart_marker_blocks=2)
    save("s422_q100_odd_45x67.jpg", textured(45, 67, 13), quality=100, subsampling=1)
    save("s422_rst2_77x130.jpg", textured(77, 130, 14), quality=60, subsampling=1,
         restart_marker_blocks=2)
    save("progressive_64x64.jpg", textured(64, 64, 12), quality=80, progressive=True)
    # progressive (SOF2: spectral selection + successive approximation, libjpeg's standard script)
    save("prog_s420_q90_600x1000.jpg", textured(600, 1000, 21), quality=90, subsampling=2,
         progressive=True)
    save("prog_s444_q85_96x128.jpg", textured(96, 128, 22), quality=85, subsampling=0,
         progressive=True)
    save("prog_s422_q75_odd_45x67.jpg", textured(45, 67, 23), quality=75, subsampling=1,
         progressive=True)
    save("prog_gray_q80_91x77.jpg", textured(91, 77, 24)[..., 0], quality=80, progressive=True)
    save("prog_s420_rst4_120x160.jpg", textured(120, 160, 25), quality=80, subsampling=2,
         progressive=True, restart_marker_blocks=4)
    derived()


def _scan_segments(data):
    """(start, end) of every SOS segment: the SOS marker up to the next marker that is not RSTn"""
    out, k = [], data.find(b"\xff\xda")
    while k >= 0:
        e = k + 2 + ((data[k + 2] << 8) | data[k + 3])
        while e + 1 < len(data) and not (data[e] == 0xFF and data[e + 1] not in (0x00, 0xFF)
                                         and not 0xD0 <= data[e + 1] <= 0xD7):
            e += 1
        out.append((k, e))
        k = data.find(b"\xff\xda", e)
    return out


def derived():
    """prog_nodc_cut_s444_96x128.jpg: prog_s444_q85_96x128.jpg without its DC scans (first and
    refinement) and without its last two scans.  Its AC 1..5 stay imprecise, but no component has
    DC data, so libjpeg 9d's smoothing_ok() is FALSE (jdcoefct.c) and it decodes WITHOUT block
    smoothing (progression warnings only): the case the decoder must accept, not reject"""
    data = (OUT / "prog_s444_q85_96x128.jpg").read_bytes()
    segs = _scan_segments(data)
    parts, prev = [], segs[0][0]
    parts.append(data[:prev])
    for k, e in segs[:-2]:
        parts.append(data[prev:k])  # the tables (DHT) defined between scans
        ns = data[k + 4]
        if data[k + 5 + 2 * ns] != 0:  # Ss > 0: an AC scan
            parts.append(data[k:e])
        prev = e
    body = b"".join(parts) + b"\xff\xd9"
    (OUT / "prog_nodc_cut_s444_96x128.jpg").write_bytes(body)
    # prog_q0_cut_s444_96x128.jpg: the same file cut before its last two scans (luma AC refinement
    # missing: imprecise), with the chroma table's Q01 set to 0.  The luma component alone would be
    # smoothed, but a zero among any component's Q00 Q01 Q10 Q20 Q11 Q02 makes smoothing_ok()
    # FALSE for the whole image: libjpeg decodes it unsmoothed
    cut = bytearray(data[:segs[-2][0]] + b"\xff\xd9")
    k = cut.find(b"\xff\xdb")
    while k >= 0:
        seg_end = k + 2 + ((cut[k + 2] << 8) | cut[k + 3])
        t = k + 4
        while t < seg_end:
            pq, tq = cut[t] >> 4, cut[t] & 15
            if tq == 1 and pq == 0:
                cut[t + 1 + 1] = 0  # zigzag index 1 = natural Q01
            t += 1 + 64 * (2 if pq else 1)
        k = cut.find(b"\xff\xdb", seg_end)
    (OUT / "prog_q0_cut_s444_96x128.jpg").write_bytes(bytes(cut))
    smoothed()
    colorspaces()
    arithmetic()
    cmyk()


def _segments(data):
    """(marker, start, end) of the marker segments before the first SOS (SOI excluded)"""
    out, i = [], 2
    while i + 4 <= len(data) and data[i] == 0xFF:
        m = data[i + 1]
        e = i + 2 + ((data[i + 2] << 8) | data[i + 3])
        out.append((m, i, e))
        if m == 0xDA:
            break
        i = e
    return out


def _recolor(src, name, ids=None, jfif=True, adobe=None):
    """`src` with its component IDs replaced (frame and every scan header), its APP0 JFIF segment
    dropped (jfif=False) and / or an APP14 Adobe segment with colour transform `adobe` added"""
    data = bytearray((OUT / src).read_bytes())
    if ids is not None:
        k = data.find(b"\xff\xc0")
        if k < 0:
            k = data.find(b"\xff\xc2")
        old = [data[k + 10 + 3 * c] for c in range(data[k + 9])]
        remap = dict(zip(old, ids))
        for c in range(len(old)):
            data[k + 10 + 3 * c] = remap[old[c]]
        k = data.find(b"\xff\xda")
        while k >= 0:
            for j in range(data[k + 4]):
                data[k + 5 + 2 * j] = remap[data[k + 5 + 2 * j]]
            k = data.find(b"\xff\xda", k + 2)
    body = bytes(data)
    if not jfif:
        for m, a, e in _segments(body):
            if m == 0xE0 and body[a + 4:a + 9] == b"JFIF\0":
                body = body[:a] + body[e:]
                break
    if adobe is not None:
        app14 = b"\xff\xee\x00\x0eAdobe\x00\x64\x00\x00\x00\x00" + bytes([adobe])
        body = body[:2] + app14 + body[2:]
    (OUT / name).write_bytes(body)


def colorspaces():
    """3-component files libjpeg 9 and libjpeg-turbo take as RGB or YCbCr by different rules
    (jdapimin.c default_decompress_parms: 9 reads the component IDs first, turbo the JFIF / Adobe
    markers first)"""
    R, G, B = 0x52, 0x47, 0x42
    # IDs 'R' 'G' 'B' with the JFIF marker: RGB for libjpeg 9, YCbCr for turbo
    _recolor("s444_q95_96x128.jpg", "cs_rgbids_jfif_s444_96x128.jpg", ids=(R, G, B))
    # IDs 'R' 'G' 'B', no marker: RGB for both (subsampled RGB, odd size)
    _recolor("s420_q75_odd_37x53.jpg", "cs_rgbids_s420_odd_37x53.jpg", ids=(R, G, B), jfif=False)
    # Adobe transform 0, IDs 1 2 3: YCbCr for libjpeg 9 (IDs first), RGB for turbo
    _recolor("s444_q95_96x128.jpg", "cs_adobe0_s444_96x128.jpg", jfif=False, adobe=0)
    # Adobe transform 0, IDs 0 1 2: RGB for both (progressive 4:2:2)
    _recolor("prog_s422_q75_odd_45x67.jpg", "cs_adobe0_ids012_prog_s422_45x67.jpg", ids=(0, 1, 2),
             jfif=False, adobe=0)
    # Adobe transform 1 with IDs 'R' 'G' 'B': RGB for libjpeg 9 (IDs), YCbCr for turbo (Adobe)
    _recolor("s422_q85_120x200.jpg", "cs_adobe1_rgbids_s422_120x200.jpg", ids=(R, G, B), jfif=False,
             adobe=1)


JPEGTRAN = Path("/opt/conda/bin/jpegtran")  # IJG libjpeg 9's jpegtran (the conda build)


def arithmetic():
    """arithmetic-coded files (SOF9 sequential / SOF10 progressive, QM-coder), losslessly
    transcoded from Huffman fixtures by libjpeg 9's jpegtran -arithmetic: what cv2.imread's
    libjpeg 9d decodes and libjpeg-turbo builds without arithmetic support refuse"""
    import subprocess

    def tran(src, name, *args):
        out = subprocess.run([str(JPEGTRAN), "-arithmetic", *args, str(OUT / src)],
                             capture_output=True, check=True).stdout
        (OUT / name).write_bytes(out)

    tran("s444_q95_96x128.jpg", "arith_s444_96x128.jpg")
    tran("s420_q75_odd_37x53.jpg", "arith_s420_odd_37x53.jpg")
    tran("s422_q85_120x200.jpg", "arith_rst_s422_120x200.jpg", "-restart", "1")
    tran("gray_q80_91x77.jpg", "arith_prog_gray_91x77.jpg", "-progressive")
    tran("s420_q75_odd_37x53.jpg", "arith_prog_s420_odd_37x53.jpg", "-progressive")
    tran("s444_q95_96x128.jpg", "arith_prog_rst_s444_96x128.jpg", "-progressive", "-restart", "1")
    # progressive arithmetic cut before its last two scans: block smoothing on arithmetic data
    _keep_scans("arith_prog_rst_s444_96x128.jpg", set(range(8)), "arith_prog_smooth_s444_96x128.jpg")


def cmyk():
    """4-component files: CMYK (Pillow writes Adobe-inverted CMYK with an APP14 transform 0) and the
    same data relabelled YCCK (transform 2), baseline and progressive, and CMYK without the Adobe
    marker (libjpeg: CMYK).  cv2.imread runs libjpeg's JCS_CMYK output through OpenCV's
    CMYK -> BGR conversion"""
    import subprocess
    rs = np.random.RandomState(31)
    y, x = np.mgrid[0:40, 0:56]
    c = np.stack([(x * 4 + rs.randint(0, 20, x.shape)) % 256, (y * 6) % 256, ((x + y) * 3) % 256,
                  64 + (x * y) % 128], -1).astype(np.uint8)
    b = io.BytesIO()
    Image.fromarray(c, "CMYK").save(b, "JPEG", quality=92)
    data = b.getvalue()
    (OUT / "cmyk_s444_40x56.jpg").write_bytes(data)
    k = data.find(b"\xff\xee")
    assert data[k + 4:k + 9] == b"Adobe" and data[k + 15] == 0
    ycck = bytearray(data)
    ycck[k + 15] = 2
    (OUT / "ycck_s444_40x56.jpg").write_bytes(bytes(ycck))
    noadobe = data[:k] + data[k + 2 + ((data[k + 2] << 8) | data[k + 3]):]
    (OUT / "cmyk_noadobe_s444_40x56.jpg").write_bytes(noadobe)
    prog = subprocess.run([str(JPEGTRAN), "-progressive", str(OUT / "ycck_s444_40x56.jpg")],
                          capture_output=True, check=True).stdout
    (OUT / "ycck_prog_s444_40x56.jpg").write_bytes(prog)


def _keep_scans(src, keep, name):
    """`src` with only the scans whose indices are in `keep` (file order), the tables between
    scans kept, ended by EOI"""
    data = (OUT / src).read_bytes()
    segs = _scan_segments(data)
    parts, prev = [data[:segs[0][0]]], segs[0][0]
    for j, (k, e) in enumerate(segs):
        parts.append(data[prev:k])
        if j in keep:
            parts.append(data[k:e])
        prev = e
    (OUT / name).write_bytes(b"".join(parts) + b"\xff\xd9")


def smoothed():
    """progressive files libjpeg 9d block-smooths (jdcoefct.c smoothing_ok TRUE: every component
    has DC data, nonzero low quantisers, and some AC 1..5 left imprecise by the last scan).  The
    fixtures' script (jpeg_simple_progression, 3 components): 0 DC first Al 1, 1 Y AC1-5 Al 2,
    2 Cr AC1-63 Al 1, 3 Cb AC1-63 Al 1, 4 Y AC6-63 Al 2, 5 Y AC1-63 refine Al 1, 6 DC refine,
    7 Cr refine, 8 Cb refine, 9 Y refine (grayscale: 0 DC, 1 AC1-5, 2 AC6-63, 3 AC refine Al 1,
    4 DC refine, 5 AC refine Al 0)"""
    # Y and Cb AC at Al 1, Cr exact (the two last scans cut)
    _keep_scans("prog_s444_q85_96x128.jpg", set(range(8)), "prog_smooth_cut_s444_96x128.jpg")
    # DC at Al 1, every AC capped (Al > 0: the 2^Al - 1 clamp), restart intervals
    _keep_scans("prog_s420_rst4_120x160.jpg", {0, 1, 2, 3}, "prog_smooth_al_s420_rst4_120x160.jpg")
    # odd 4:2:2 (edge blocks, the 16x8 chroma IDCT), refinements missing
    _keep_scans("prog_s422_q75_odd_45x67.jpg", set(range(6)), "prog_smooth_s422_odd_45x67.jpg")
    # chroma AC never sent (coef_bits -1: estimates without a cap), luma AC 1-5 at Al 2
    _keep_scans("prog_s444_q85_96x128.jpg", {0, 1}, "prog_smooth_dconly_s444_96x128.jpg")
    # grayscale, DC and the AC refinement missing
    _keep_scans("prog_gray_q80_91x77.jpg", {0, 1, 2, 3}, "prog_smooth_gray_91x77.jpg")


if __name__ == "__main__":
    import sys
    derived() if sys.argv[1:] == ["--derived"] else main()
