"""Image loading for the drop-in path: cv2.imread semantics (BGR uint8 HxWx3).

The reference reads every image with cv2.imread (lib/model/test.py:191,
lib/roi_data_layer/minibatch.py:85), i.e. OpenCV 3.4.2 over IJG libjpeg 9d (requirements.txt:74,
89).  `imread` uses OpenCV when it is importable.  Without it, a JPEG is decoded by the GPU decoder
(`imread_gpu`: bit-exact with libjpeg 9d) and returned as a host array -- never by PIL, whose
libjpeg-turbo differs from 9d by up to tens of LSB on subsampled files; a JPEG the GPU decoder
does not take raises IdnError.  Other (lossless) formats go through PIL, flipped to BGR.

`imread_gpu` is the GPU decode front-end: JPEG files are decoded on the
device (idn_jpeg_decode_u8), bit-exact with the reference's pinned IJG libjpeg 9d by default or
with libjpeg-turbo (mode="turbo"), images of one size in one launch; files the decoder does not
take raise IdnError (no CPU fallback inside the product).  Like OpenCV 3.4.2's imread, each JPEG
is turned by its EXIF orientation (APP1 IFD0 tag 0x0112: flips / transposes; idn_jpeg_orientation)
unless orientation=False (IMREAD_IGNORE_ORIENTATION).  PNG and the other lossless formats never
carry it in the form OpenCV 3.4.2's EXIF reader walks (it reads JPEG markers), so `_imread_pil`
leaves them as stored.
"""
from __future__ import annotations

import numpy as np


def imread(path) -> np.ndarray:
    """cv2.imread(path) (IMREAD_COLOR) as a host uint8 BGR HxWx3 array."""
    try:
        import cv2
    except ImportError:
        cv2 = None
    if cv2 is not None:
        im = cv2.imread(str(path))
        if im is None:
            raise FileNotFoundError(path)
        return im
    with open(path, "rb") as f:
        head = f.read(3)
    if head[:2] == b"\xff\xd8":  # JPEG: the libjpeg 9d decode, on the GPU
        return imread_gpu([path])[0].cpu().numpy()
    return _imread_pil(path)


def _imread_pil(path) -> np.ndarray:
    """a lossless format through PIL, as OpenCV's decoders return it with IMREAD_COLOR: 8-bit BGR,
    alpha dropped, palettes expanded.  Samples deeper than 8 bits keep their high byte, as
    grfmt_png.cpp's png_set_strip_16 does (PIL's own 16-bit grayscale -> RGB conversion would clip
    them at 255 instead); PIL already unpacks 16-bit RGB(A) to its high bytes."""
    from PIL import Image
    with Image.open(path) as im:
        if im.mode in ("I;16", "I;16B", "I;16L", "I"):
            g = np.asarray(im).astype(np.int64)
            if im.mode == "I" and g.max(initial=0) > 0xFFFF:
                raise ValueError(f"{path}: 32-bit samples are not an OpenCV IMREAD_COLOR input")
            g = (g >> 8).astype(np.uint8)
            return np.ascontiguousarray(np.repeat(g[..., None], 3, -1))
        rgb = np.asarray(im.convert("RGB"))
    return np.ascontiguousarray(rgb[..., ::-1])


def imread_gpu(paths, mode: str = "libjpeg9", orientation: bool = True):
    """cv2.imread for a list of JPEG paths, decoded on the GPU: a list of (h, w, 3) uint8 BGR
    device tensors in input order, each turned by its EXIF orientation (orientation=False:
    IMREAD_IGNORE_ORIENTATION); files of the same output size share one decode launch."""
    from . import ops
    datas = []
    for p in paths:
        with open(p, "rb") as f:
            datas.append(f.read())
    groups = {}
    for i, d in enumerate(datas):
        groups.setdefault(ops.jpeg_info(d, orientation)[:2], []).append(i)
    out = [None] * len(datas)
    for idx in groups.values():
        dec = ops.jpeg_decode([datas[i] for i in idx], mode=mode, orientation=orientation)
        for k, i in enumerate(idx):
            out[i] = dec[k]
    return out


class ImageReader:
    """The test loop's image reads (lib/model/test.py:189-191: `for i in range(num_images):
    img = cv2.imread(imdb.image_path_at(i))`) with read-ahead: reader[i] is
    imread_gpu([paths[i]])[0], but the files are decoded `batch` at a time (one decode launch per
    window of same-size files), and while the caller works on the images of window b, window
    b + 1 decodes on a side stream from a worker thread.  A single file's decode is latency-bound
    (its entropy passes keep ~16 waves busy for ~1.3 ms while the host waits on their
    convergence flags) and a window of 8 takes about as long as one, so read-ahead turns the
    decode from the loop's largest stage into one hidden behind the current image's noise,
    wavelet and blob work and its copy to the host.  Results are those of imread_gpu (the decode
    is per file; batching does not change a byte); access is expected in order (an index outside
    the windows in flight decodes its own window on demand).

        reader = ImageReader([imdb.image_path_at(i) for i in range(num_images)])
        for i in range(num_images):
            im = apply_noise(reader[i], noise, decode="gpu", as_tensor=True)
            ...
    """

    def __init__(self, paths, mode: str = "libjpeg9", orientation: bool = True, prefetch: bool = True,
                 batch: int = 8):
        import concurrent.futures
        import torch
        if batch < 1:
            raise ValueError("ImageReader: batch must be >= 1")
        self.paths = [str(p) for p in paths]
        self.mode, self.orientation, self.batch = mode, orientation, int(batch)
        self._dev = torch.cuda.current_device()
        self._side = torch.cuda.Stream(self._dev)
        self._pool = concurrent.futures.ThreadPoolExecutor(1) if prefetch else None
        self._pending = {}  # window -> future of (images, event)
        self._win = None    # (window, images, event) being read

    def __len__(self):
        return len(self.paths)

    def _decode(self, b):
        import torch
        lo = b * self.batch
        with torch.cuda.device(self._dev), torch.cuda.stream(self._side):
            ims = imread_gpu(self.paths[lo:lo + self.batch], self.mode, self.orientation)
            ev = torch.cuda.Event()
            ev.record(self._side)
        return ims, ev

    def __getitem__(self, i: int):
        import torch
        if not 0 <= i < len(self.paths):
            raise IndexError(i)
        b = i // self.batch
        if self._win is None or self._win[0] != b:
            fut = self._pending.pop(b, None)
            ims, ev = fut.result() if fut is not None else self._decode(b)
            self._win = (b, ims, ev)
            if (self._pool is not None and (b + 1) * self.batch < len(self.paths)
                    and b + 1 not in self._pending):
                self._pending[b + 1] = self._pool.submit(self._decode, b + 1)
        _, ims, ev = self._win
        im = ims[i - b * self.batch]
        cur = torch.cuda.current_stream(self._dev)
        cur.wait_event(ev)
        im.record_stream(cur)  # decoded on the side stream, used on the caller's
        return im

    def close(self):
        for f in self._pending.values():
            f.result()
        self._pending.clear()
        self._win = None
        if self._pool is not None:
            self._pool.shutdown(wait=True)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
