"""Expected cv2.imread pixels of damaged JPEG files, as the reference's pinned libjpeg 9d makes them.

The damaged files are the recipes of tests/golden/jpeg_damage.py applied to the committed fixture
files (files cut short, bit errors, bad Huffman codes, lost / renumbered restart markers, stray
markers).  libjpeg decodes them with warnings only (JWRN_HIT_MARKER, JWRN_HUFF_BAD_CODE,
JWRN_MUST_RESYNC ...) and returns an image; cv2.imread returns the same pixels.  Decoded here by
`/opt/conda/bin/python3.9`'s Pillow 8.4.0 over `/opt/conda/lib/libjpeg.so.9` (9d), as
tests/golden/make_jpeg9_fixtures.py does for the intact files.

Written: tests/golden/jpeg9_damaged.json (per case: shape, sha256 of the BGR array, channel sums)
and tests/golden/jpeg9_damaged.npz (per case the row sums per channel, to locate a divergence).

  /opt/conda/bin/python3.9 tests/golden/make_jpeg_damaged.py
"""
import hashlib
import io
import json
import sys
from pathlib import Path

import numpy as np
from PIL import Image, features

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
import jpeg_damage  # noqa: E402


def bgr(data: bytes):
    with Image.open(io.BytesIO(data)) as im:
        if im.mode == "CMYK":  # as make_jpeg9_fixtures.bgr: libjpeg's CMYK through OpenCV's formula
            c = 255 - np.asarray(im).astype(np.int64)
            k = c[..., 3]
            return np.ascontiguousarray(np.stack(
                [k - (((255 - c[..., j]) * k) >> 8) for j in (2, 1, 0)], -1).astype(np.uint8))
        a = np.asarray(im.convert("RGB"))
    return np.ascontiguousarray(a[..., ::-1])


def main():
    ver = features.version("jpg")
    if not ver or not ver.startswith("9"):
        raise SystemExit(f"needs Pillow linked with IJG libjpeg 9 (found {ver!r}): "
                         "run under /opt/conda/bin/python3.9")
    meta, arrays = {"libjpeg": ver, "cases": {}}, {}
    for case in jpeg_damage.cases():
        k = jpeg_damage.key(case)
        data = jpeg_damage.damage((HERE / "jpeg" / case[0]).read_bytes(), case[1], case[2])
        a = bgr(data)
        rec = {"shape": list(a.shape), "sha256": hashlib.sha256(a.tobytes()).hexdigest(),
               "sums": [int(a[..., c].astype(np.int64).sum()) for c in range(3)]}
        arrays[k] = a.astype(np.int64).sum(axis=1).astype(np.uint32)  # per row and channel
        meta["cases"][k] = rec
    np.savez_compressed(HERE / "jpeg9_damaged.npz", **arrays)
    (HERE / "jpeg9_damaged.json").write_text(json.dumps(meta, indent=1) + "\n")
    print(len(meta["cases"]), "cases")


if __name__ == "__main__":
    main()
