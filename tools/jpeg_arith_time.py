"""Decode time of arithmetic-coded files (tools only): a synthetic 600x1000 q90 file converted by
libjpeg 9's jpegtran (/opt/conda/bin/jpegtran -arithmetic, sequential and progressive), median of
synchronous calls.  python tools/jpeg_arith_time.py [--iters 5]"""
import argparse
import io
import statistics
import subprocess
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    x = bench.synth_batch(torch, 1, torch.device("cuda", 0), seed=3).cpu().numpy()
    b = io.BytesIO()
    Image.fromarray(x[0][..., ::-1]).save(b, "JPEG", quality=90, subsampling=2)
    base = b.getvalue()
    for name, args in [("arith sequential", ["-arithmetic"]),
                       ("arith progressive", ["-arithmetic", "-progressive"]),
                       ("arith sequential, restart per row", ["-arithmetic", "-restart", "1"])]:
        f = subprocess.run(["/opt/conda/bin/jpegtran", *args], input=base, capture_output=True,
                           check=True).stdout
        ops.jpeg_decode([f])
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.iters):
            t = time.perf_counter()
            ops.jpeg_decode([f])
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t) * 1e3)
        print(f"{name}: {len(f)} bytes, {statistics.median(ts):.2f} ms", flush=True)


if __name__ == "__main__":
    main()
