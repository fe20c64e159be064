"""JPEG decode time per decoder path (tools only): median wall time of synchronous calls for
  baseline    one synthetic 600x1000 q90 4:2:0 file (the chunked decoder), and a batch of 64
  restart     the same image with a restart marker every MCU row (one thread per interval)
  progressive the same image progressive (the scan path), and a batch of 16
  python tools/jpeg_paths_time.py [--iters 40]"""
import argparse
import io
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "image-denoising_amd"))
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402
from PIL import Image  # noqa: E402

import bench  # noqa: E402
from idn import ops  # noqa: E402


def med(files, iters):
    ops.jpeg_decode(files)
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        t = time.perf_counter()
        ops.jpeg_decode(files)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=40)
    a = ap.parse_args()
    x = bench.synth_batch(torch, 1, torch.device("cuda", 0), seed=3).cpu().numpy()
    im = Image.fromarray(x[0][..., ::-1])
    files = {}
    for name, kw in [("baseline", {}), ("restart", {"restart_marker_rows": 1}),
                     ("progressive", {"progressive": True})]:
        b = io.BytesIO()
        im.save(b, "JPEG", quality=90, subsampling=2, **kw)
        files[name] = b.getvalue()
    for name, n in [("baseline", 1), ("baseline", 64), ("restart", 1), ("restart", 64),
                    ("progressive", 1), ("progressive", 16)]:
        print(f"{name} x{n} {med([files[name]] * n, a.iters):.4f} ms", flush=True)


if __name__ == "__main__":
    main()
