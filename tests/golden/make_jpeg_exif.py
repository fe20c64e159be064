"""Fixtures for cv2.imread's EXIF orientation step (OpenCV 3.4.2 loadsave.cpp ApplyExifOrientation;
call sites /root/reference/lib/model/test.py:191, lib/roi_data_layer/minibatch.py:85).

Files (tests/golden/jpeg_exif/):
* Pillow-written, one per orientation 1..8 of a baseline odd 4:2:0 file and of a progressive odd
  4:2:2 file, plus grayscale, restart-interval and 600x1000 files: Pillow puts its EXIF block
  ("Exif\\0\\0", little-endian TIFF, IFD0 with Orientation) in an APP1 after the JFIF APP0, and the
  entropy-coded data do not depend on it.
* derived from the orientation-1 baseline file by splicing hand-built APP1 blocks in: big-endian
  TIFF, extra tags before / after Orientation, an XMP APP1 ahead of the EXIF one, out-of-range
  values, a truncated IFD, a malformed string tag, duplicate tags, a bad TIFF mark, a too-short
  APP1, EXIF after DQT / COM.  Their orientation is what OpenCV 3.4.2's exif.cpp gives
  (restated, cv2 is not importable here): "orientation" in the JSON, next to Pillow's own reading
  ("pil_orientation", None where Pillow reads none).

Expected pixels: the reference's pinned IJG libjpeg 9d decode (this script runs under
/opt/conda/bin/python3.9, whose Pillow 8.4.0 links libjpeg 9d) turned by that orientation with
Pillow's own Image.transpose methods (2 FLIP_LEFT_RIGHT, 3 ROTATE_180, 4 FLIP_TOP_BOTTOM,
5 TRANSPOSE, 6 ROTATE_270, 7 TRANSVERSE, 8 ROTATE_90 -- the same eight images OpenCV's flip /
transpose sequence makes), so the geometry is not the oracle's own code.  Written:
  tests/golden/jpeg_exif.npz   full BGR arrays of the small files, 32x32 crops of the large one
  tests/golden/jpeg_exif.json  per file: orientation, pil_orientation, shape, sha256, sums, crops

  /opt/conda/bin/python3.9 tests/golden/make_jpeg_exif.py
"""
import hashlib
import io
import json
import struct
from pathlib import Path

import numpy as np
from PIL import Image, features

HERE = Path(__file__).resolve().parent
OUT = HERE / "jpeg_exif"
FULL_LIMIT = 130 * 200


def textured(h, w, seed):
    rs = np.random.RandomState(seed)
    y, x = np.mgrid[0:h, 0:w]
    base = 128 + 60 * np.sin(x / 13.0 + seed) * np.cos(y / 19.0) + rs.normal(0, 18, (h, w))
    # an asymmetric ramp, so every flip / transpose of the image differs
    base = base + 0.6 * x - 0.4 * y
    img = np.stack([base, np.roll(base, 5, 1) * 0.8 + 30, 255 - base], -1)
    return np.clip(img, 0, 255).astype(np.uint8)


def exif_bytes(orient):
    ex = Image.Exif()
    ex[0x0112] = orient
    return ex.tobytes()


def encode(arr, orient=None, **kw):
    b = io.BytesIO()
    if orient is not None:
        kw["exif"] = exif_bytes(orient)
    Image.fromarray(arr).save(b, "JPEG", **kw)
    return b.getvalue()


# ---- hand-built EXIF blocks ---------------------------------------------------------------------
def tiff(entries, big=False, ifd_off=8, mark=42, extra=b"", count=None):
    """a TIFF block: header, IFD0 of (tag, type, count, value-bytes-or-int) entries, extra data"""
    e = ">" if big else "<"
    out = (b"MM" if big else b"II") + struct.pack(e + "HI", mark, ifd_off)
    out += b"\0" * (ifd_off - 8)
    out += struct.pack(e + "H", len(entries) if count is None else count)
    for tag, typ, cnt, val in entries:
        if isinstance(val, bytes):
            v = val.ljust(4, b"\0")
        elif typ == 3:  # SHORT: left-justified in the 4-byte value field
            v = struct.pack(e + "HH", val, 0)
        else:
            v = struct.pack(e + "I", val)
        out += struct.pack(e + "HHI", tag, typ, cnt) + v
    out += struct.pack(e + "I", 0) + extra
    return out


def app1(payload, ident=b"Exif\0\0"):
    body = ident + payload
    return b"\xff\xe1" + struct.pack(">H", len(body) + 2) + body


def insert_after(data, marker, seg):
    """seg after the first segment with this marker code (SOI: right after the file's first 2 bytes)"""
    if marker == 0xD8:
        return data[:2] + seg + data[2:]
    k = data.find(bytes([0xFF, marker]))
    end = k + 2 + (data[k + 2] << 8 | data[k + 3])
    return data[:end] + seg + data[end:]


def derived(plain):
    """(name, file bytes, OpenCV 3.4.2's orientation) built from an orientation-less file"""
    o6 = (0x0112, 3, 1, 6)
    cases = []
    add = lambda name, seg, o, where=0xE0: cases.append((name, insert_after(plain, where, seg), o))
    add("mm_o6", app1(tiff([o6], big=True)), 6)
    # Make (a 12-byte string stored past the IFD) then Orientation, big-endian
    make_off = 8 + 2 + 2 * 12 + 4
    add("mm_make_o7", app1(tiff([(0x010F, 2, 12, make_off), (0x0112, 3, 1, 7)], big=True,
                                extra=b"IDN-CAMERA!\0")), 7)
    # resolution (a rational at an offset) and a short string held in the value field
    res_off = 8 + 2 + 3 * 12 + 4
    add("ii_res_str_o5", app1(tiff([(0x011A, 5, 1, res_off), (0x0131, 2, 4, b"idn\0"),
                                    (0x0112, 3, 1, 5)], extra=struct.pack("<II", 72, 1))), 5)
    # an XMP APP1 first: OpenCV takes it as the EXIF block (no TIFF mark: no orientation); Pillow
    # finds the real one after it
    xmp = app1(b"<x:xmpmeta xmlns:x='adobe:ns:meta/'/>", ident=b"http://ns.adobe.com/xap/1.0/\0")
    add("xmp_first_o6", xmp + app1(tiff([o6])), 1)
    add("o9", app1(tiff([(0x0112, 3, 1, 9)])), 1)
    add("o0", app1(tiff([(0x0112, 3, 1, 0)])), 1)
    add("trunc_ifd_o6", app1(tiff([o6], count=30)), 1)  # the 3rd entry lies past the data
    add("bad_make_after_o6", app1(tiff([o6, (0x010F, 2, 40, 5000)])), 1)  # string past the data
    add("bad_res_after_o8", app1(tiff([(0x0112, 3, 1, 8), (0x011B, 5, 1, 1 << 20)])), 1)
    add("dup_o3_o6", app1(tiff([(0x0112, 3, 1, 3), o6])), 3)
    add("unknown_tags_o2", app1(tiff([(0x9000, 7, 4, b"0230"), (0x0112, 3, 1, 2),
                                      (0x8769, 4, 1, 0)])), 2)  # ExifIFD pointer: not followed
    add("bad_mark_o6", app1(tiff([o6], mark=43)), 1)
    add("app1_len6", b"\xff\xe1\x00\x06Exif", 1)
    add("after_dqt_o5", app1(tiff([(0x0112, 3, 1, 5)])), 5, where=0xDB)
    add("after_com_o8", b"\xff\xfe\x00\x07idn!\0" + app1(tiff([(0x0112, 3, 1, 8)])), 8)
    add("ifd_offset_o4", app1(tiff([(0x0112, 3, 1, 4)], ifd_off=20)), 4)
    return cases


PIL_T = {2: Image.FLIP_LEFT_RIGHT, 3: Image.ROTATE_180, 4: Image.FLIP_TOP_BOTTOM,
         5: Image.TRANSPOSE, 6: Image.ROTATE_270, 7: Image.TRANSVERSE, 8: Image.ROTATE_90}


def expected(data, orient):
    with Image.open(io.BytesIO(data)) as im:
        im = im.convert("RGB")
        if orient in PIL_T:
            im = im.transpose(PIL_T[orient])
        a = np.asarray(im)
    return np.ascontiguousarray(a[..., ::-1])


def pil_orientation(data):
    with Image.open(io.BytesIO(data)) as im:
        return im.getexif().get(0x0112)


def main():
    ver = features.version("jpg")
    if not ver or not ver.startswith("9"):
        raise SystemExit(f"needs Pillow linked with IJG libjpeg 9 (found {ver!r}): "
                         "run under /opt/conda/bin/python3.9")
    OUT.mkdir(exist_ok=True)
    files = {}
    a420, a422 = textured(37, 53, 31), textured(45, 67, 32)
    for o in range(1, 9):
        files[f"s420_o{o}_37x53.jpg"] = (encode(a420, o, quality=75, subsampling=2), o)
        files[f"prog_s422_o{o}_45x67.jpg"] = (encode(a422, o, quality=80, subsampling=1,
                                                     progressive=True), o)
    files["gray_o6_29x41.jpg"] = (encode(textured(29, 41, 33)[..., 0], 6, quality=85), 6)
    files["gray_o3_29x41.jpg"] = (encode(textured(29, 41, 33)[..., 0], 3, quality=85), 3)
    files["s420_rstrow_o8_120x160.jpg"] = (encode(textured(120, 160, 34), 8, quality=80,
                                                  subsampling=2, restart_marker_rows=1), 8)
    files["s420_o6_600x1000.jpg"] = (encode(textured(600, 1000, 35), 6, quality=90,
                                            subsampling=2), 6)
    plain = encode(a420, None, quality=75, subsampling=2)
    for name, data, o in derived(plain):
        files[f"s420_{name}_37x53.jpg"] = (data, o)
    meta, arrays = {"libjpeg": ver, "files": {}}, {}
    for name, (data, o) in sorted(files.items()):
        (OUT / name).write_bytes(data)
        a = expected(data, o)
        h, w = a.shape[:2]
        rec = {"orientation": o, "pil_orientation": pil_orientation(data), "shape": list(a.shape),
               "sha256": hashlib.sha256(a.tobytes()).hexdigest(),
               "sums": [int(a[..., c].astype(np.int64).sum()) for c in range(3)]}
        if h * w <= FULL_LIMIT:
            arrays[name] = a
            rec["full"] = True
        else:
            crops = [(0, 0), (h - 32, w - 32), (h // 2 - 16, w // 2 - 16), (17, w - 51), (h - 45, 13)]
            rec["crops"] = crops
            for k, (y, x) in enumerate(crops):
                arrays[f"{name}:crop{k}"] = a[y:y + 32, x:x + 32]
        meta["files"][name] = rec
    np.savez_compressed(HERE / "jpeg_exif.npz", **arrays)
    (HERE / "jpeg_exif.json").write_text(json.dumps(meta, indent=1) + "\n")


if __name__ == "__main__":
    main()
