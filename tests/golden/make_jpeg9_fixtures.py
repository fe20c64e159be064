"""Expected pixels of cv2.imread for the JPEG fixtures, as the reference's pinned decoder makes them.

The reference pins IJG libjpeg 9d (`/root/reference/requirements.txt:74`, `jpeg=9d`) under
OpenCV 3.4.2 (`requirements.txt:89,121,141`); cv2.imread (`lib/model/test.py:191`,
`lib/roi_data_layer/minibatch.py:85`) decodes with that library's defaults (ISLOW, fancy
upsampling -> libjpeg >= 7 scales the subsampled chroma IDCT to 16x16 / 16x8, see
oracle/jpeg9.py) into JCS_RGB and swaps to BGR.  In this container `/opt/conda/bin/python3.9`'s
Pillow 8.4.0 links `/opt/conda/lib/libjpeg.so.9` (9d, reported as "9.0"); its RGB decode of each
fixture file, flipped to BGR, is the expected output.  (The system Python's Pillow 12.2 links
libjpeg-turbo, which decodes every subsampled file differently.)

Written (the GPU box has no libjpeg 9, so the expected pixels travel as data):
  tests/golden/jpeg9.npz   full BGR arrays of the small files; 32x32 crops of the large ones
  tests/golden/jpeg9.json  per file: shape, sha256 of the full BGR array, per-channel sums, crops

  /opt/conda/bin/python3.9 tests/golden/make_jpeg9_fixtures.py
"""
import hashlib
import json
from pathlib import Path

import numpy as np
from PIL import Image, features

HERE = Path(__file__).resolve().parent
JPEG = HERE / "jpeg"
FULL_LIMIT = 130 * 200  # files up to this many pixels are stored whole


def bgr(path):
    with Image.open(path) as im:
        if im.mode == "CMYK":
            # Pillow reads libjpeg's JCS_CMYK output inverted ("CMYK;I"): undo that, then apply
            # OpenCV's icvCvt_CMYK2BGR_8u_C4C3R (grfmt_jpeg.cpp's 4-component path), which is
            # restated from the published OpenCV source (cv2 is not importable here)
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
    meta, arrays = {"libjpeg": ver, "files": {}}, {}
    for p in sorted(JPEG.glob("*.jpg")):
        a = bgr(p)
        h, w = a.shape[:2]
        rec = {"shape": list(a.shape), "sha256": hashlib.sha256(a.tobytes()).hexdigest(),
               "sums": [int(a[..., c].astype(np.int64).sum()) for c in range(3)]}
        if h * w <= FULL_LIMIT:
            arrays[p.name] = a
            rec["full"] = True
        else:
            crops = [(0, 0), (h - 32, w - 32), (h // 2 - 16, w // 2 - 16), (17, w - 51),
                     (h - 45, 13)]
            rec["crops"] = crops
            for k, (y, x) in enumerate(crops):
                arrays[f"{p.name}:crop{k}"] = a[y:y + 32, x:x + 32]
        meta["files"][p.name] = rec
    np.savez_compressed(HERE / "jpeg9.npz", **arrays)
    (HERE / "jpeg9.json").write_text(json.dumps(meta, indent=1) + "\n")


if __name__ == "__main__":
    main()
