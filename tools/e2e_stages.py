"""Per-stage breakdown of bench.py's detect_e2e step (tools only): the reference's per-image
test_net body, lib/model/test.py:189-191 (cv2.imread), 1678-1684 (gaussian noise, float64),
1787-1811 (the bior1.5 wavelet hook), 85-90 (_get_blobs, fed to the net from host memory).

  python tools/e2e_stages.py [--iters 200] [--out file.json]

Each stage is bracketed by torch.cuda.synchronize() and timed on the host clock (medians over the
iterations); the whole step is also timed without the inner synchronisations, as the bench does, and the loop
over eight distinct files with read-ahead (idn.io.ImageReader), as bench.py's detect_e2e_pipelined."""
import argparse
import json
import os
import statistics
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "image-denoising_amd"))
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from idn import blobs, detect_blob, io as idn_io, ops  # noqa: E402

TIMES = {}


def timed(name, fn):
    def wrap(*a, **k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn(*a, **k)
        torch.cuda.synchronize()
        TIMES.setdefault(name, []).append((time.perf_counter() - t0) * 1e3)
        return r
    return wrap


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    x = bench.synth_batch(torch, 1, torch.device("cuda", 0), seed=3)
    d = tempfile.mkdtemp(prefix="idn_e2e_")
    path = os.path.join(d, "im.jpg")
    from PIL import Image
    Image.fromarray(x[0].cpu().numpy()[..., ::-1]).save(path, "JPEG", quality=90, subsampling=2)

    def step():
        im = detect_blob.apply_noise(path, "gaussian_wavelet_var0.1", mode="test_v0",
                                     decode="gpu", as_tensor=True)
        detect_blob._get_blobs(im)

    for _ in range(20):
        step()
    torch.cuda.synchronize()
    # the whole step as the bench times it (no inner synchronisation)
    t0 = time.perf_counter()
    for _ in range(args.iters):
        step()
    torch.cuda.synchronize()
    whole = (time.perf_counter() - t0) * 1e3 / args.iters
    # the loop with read-ahead (idn.io.ImageReader: windows of 8 files, the next one decoded on a
    # side stream while this window's images run)
    paths = []
    for j in range(8):
        pj = os.path.join(d, f"ra{j}.jpg")
        Image.fromarray(np.roll(x[0].cpu().numpy()[..., ::-1], 37 * j, axis=1)).save(
            pj, "JPEG", quality=90, subsampling=2)
        paths.append(pj)
    reader = idn_io.ImageReader(paths * (args.iters // 8 + 8), batch=8)

    def step_ra(k):
        im = detect_blob.apply_noise(reader[k], "gaussian_wavelet_var0.1", mode="test_v0",
                                     decode="gpu", as_tensor=True)
        detect_blob._get_blobs(im)

    for k in range(32):
        step_ra(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(32, 32 + args.iters):
        step_ra(k)
    torch.cuda.synchronize()
    read_ahead = (time.perf_counter() - t0) * 1e3 / args.iters
    reader.close()
    # stages
    orig = (idn_io.imread_gpu, ops.random_noise_ycc, ops.denoise_wavelet, ops.blob,
            blobs.im_list_to_blob, ops.random_noise)
    idn_io.imread_gpu = timed("decode (file read + jpeg_info + GPU decode)", orig[0])
    ops.random_noise_ycc = timed("noise (gaussian, float64 out, fused colour range)", orig[1])
    ops.random_noise = timed("noise (unfused)", orig[5])
    ops.denoise_wavelet = timed("wavelet (bior1.5 on float64)", orig[2])
    ops.blob = timed("blob (prep_im_for_blob: u8 -> float32 - means)", orig[3])
    ilb = orig[4]

    def im_list_to_blob(ims, as_tensor=False):
        b = timed("im_list_to_blob (pad + copy, device)", ilb)(ims, as_tensor=True)
        return b if as_tensor else timed("D2H (blob to host numpy, pinned)", blobs._to_host)(b)
    blobs.im_list_to_blob = im_list_to_blob
    detect_blob._blob.im_list_to_blob = im_list_to_blob
    TIMES.clear()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        step()
    torch.cuda.synchronize()
    synced = (time.perf_counter() - t0) * 1e3 / args.iters
    rec = {"ms_per_image_unsynced": round(whole, 4), "ms_per_image_read_ahead": round(read_ahead, 4),
           "ms_per_image_with_stage_syncs": round(synced, 4),
           "stages_ms_median": {k: round(statistics.median(v), 4) for k, v in TIMES.items()},
           "iters": args.iters}
    rec["stages_sum_ms"] = round(sum(rec["stages_ms_median"].values()), 4)
    rec["host_overhead_ms"] = round(synced - rec["stages_sum_ms"], 4)
    s = json.dumps(rec, indent=1)
    print(s)
    if args.out:
        Path(args.out).write_text(s + "\n")


if __name__ == "__main__":
    main()
