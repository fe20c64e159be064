"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by the product path).

CPU restatement of the EXIF orientation step of `cv2.imread(path)` in the reference's pinned
OpenCV 3.4.2 (`/root/reference/requirements.txt:89`; call sites `lib/model/test.py:191`,
`lib/roi_data_layer/minibatch.py:85`).  OpenCV is a third-party library absent from
/root/reference and not importable here; its published source is restated [recalled]:

  loadsave.cpp  imread: unless IMREAD_IGNORE_ORIENTATION, ApplyExifOrientation(filename, img):
                orientation 2 flip(1), 3 flip(-1), 4 flip(0), 5 transpose, 6 transpose + flip(1),
                7 transpose + flip(-1), 8 transpose + flip(0); anything else leaves the image
  exif.cpp      ExifReader::getExif: walks the stream two bytes at a time (the 0xFF is not
                checked); SOF0 SOF2 DHT DQT DRI SOS RST0-7 APP0 APP2-15 COM are skipped by their
                length field (a length < 2 is a parse error), SOI / EOI have none, the FIRST APP1
                is the EXIF block whatever its identifier (length <= 6: error; the data are the
                length - 6 bytes after the 6-byte identifier slot, zero-filled past the end of
                the file), any other code ends the search.  parseExif: "II" little-endian, else
                big-endian reads ("MM", other equal pairs, unequal bytes); u16 at 2 must be 42;
                IFD0 at the u32 at 4; every entry of a tag it knows reads its value (strings,
                rationals, u16s), any offset past the data aborts the whole parse; the first
                entry of a tag wins; Orientation (0x0112) = the u16 at entry + 8.  32-bit offset
                arithmetic wraps like exif.cpp's uint32_t.

The device restatement is `jpg_exif_orientation` in image-denoising_amd/csrc/jpeg.hip; tests check
the two against each other and against Pillow's own reading of the tag (Image.getexif)."""
import numpy as np

_SKIP = {0xC0, 0xC2, 0xC4, 0xDB, 0xDD, 0xDA, 0xFE, 0xE0} | set(range(0xD0, 0xD8)) | set(range(0xE2, 0xF0))
_STRINGS = {0x010E, 0x010F, 0x0110, 0x0131, 0x0132, 0x8298}
_RATIONALS = {0x011A: 1, 0x011B: 1, 0x013E: 2, 0x013F: 6, 0x0211: 3, 0x0214: 6}
_U16 = {0x0128, 0x0213}
M32 = 0xFFFFFFFF


class _Bad(Exception):
    """exif.cpp's ExifParsingError"""


def _app1(data: bytes):
    """getExif's marker walk: the APP1 data block, or None (no EXIF or a parse error)"""
    i, n = 0, len(data)
    while True:
        if i + 2 > n:
            return None
        m = data[i + 1]
        i += 2

        def field():
            nonlocal i
            if i + 2 > n:
                i = n
                return 0
            v = data[i] << 8 | data[i + 1]
            i += 2
            return v
        if m in _SKIP:
            skip = field()
            if skip < 2:
                return None
            i += skip - 2
        elif m in (0xD8, 0xD9):
            continue
        elif m == 0xE1:
            size = field()
            if size <= 6:
                return None
            i += 6
            block = bytearray(size - 6)
            part = data[i:i + size - 6]
            block[:len(part)] = part
            return bytes(block)
        else:
            return None


def orientation(data: bytes) -> int:
    """the orientation OpenCV 3.4.2's imread applies to JPEG file `data` (1 = none)"""
    d = _app1(data)
    if d is None:
        return 1
    n = len(d)
    intel = not (n > 1 and d[0] != d[1]) and d[0] == ord("I")

    def u16(o):
        if o + 1 >= n:
            raise _Bad
        return d[o] | d[o + 1] << 8 if intel else d[o] << 8 | d[o + 1]

    def u32(o):
        if o + 3 >= n:
            raise _Bad
        b = d[o:o + 4]
        return int.from_bytes(b, "little" if intel else "big")
    try:
        if u16(2) != 0x2A:
            return 1
        off = u32(4)
        nent = u16(off)
        off = (off + 2) & M32
        orient = None
        for _ in range(nent):
            tag = u16(off)
            if tag in _STRINGS:
                size = u32(off + 4)
                doff = u32(off + 8) if size > 4 else 8
                if doff > n or ((doff + size) & M32) > n:
                    raise _Bad
            elif tag == 0x0112:
                v = u16(off + 8)
                if orient is None:
                    orient = v
            elif tag in _RATIONALS:
                r = u32(off + 8)
                for _k in range(_RATIONALS[tag]):
                    u32(r)
                    u32((r + 4) & M32)
                    r = (r + 8) & M32
            elif tag in _U16:
                u16(off + 8)
            off = (off + 12) & M32
    except _Bad:
        return 1
    return orient if orient is not None and 1 <= orient <= 8 else 1


def apply(img: np.ndarray, orient: int) -> np.ndarray:
    """ApplyExifOrientation's cv::flip / cv::transpose sequence on an (H, W, C) array"""
    if orient in (5, 6, 7, 8):
        img = img.transpose(1, 0, 2)
    flip = {2: 1, 3: -1, 4: 0, 6: 1, 7: -1, 8: 0}.get(orient)
    if flip == 1:
        img = img[:, ::-1]
    elif flip == 0:
        img = img[::-1]
    elif flip == -1:
        img = img[::-1, ::-1]
    return np.ascontiguousarray(img)
