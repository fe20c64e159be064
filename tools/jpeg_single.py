"""Decode one synthetic 600x1000 q90 4:2:0 file (or a batch of copies) repeatedly (tools only;
for kernel traces):
  python tools/jpeg_single.py [--iters 20] [--chunk 0] [--batch 1] [--progressive]"""
import argparse
import io
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "image-denoising_amd"))
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402
from PIL import Image  # noqa: E402

import bench  # noqa: E402
from idn import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--chunk", type=int, default=0)
ap.add_argument("--batch", type=int, default=1)
ap.add_argument("--progressive", action="store_true")
a = ap.parse_args()
x = bench.synth_batch(torch, a.batch, torch.device("cuda", 0), seed=3).cpu().numpy()
files = []
for im in x:
    b = io.BytesIO()
    Image.fromarray(im[..., ::-1]).save(b, "JPEG", quality=90, subsampling=2,
                                        progressive=a.progressive)
    files.append(b.getvalue())
print("file bytes", len(files[0]))
for _ in range(a.iters):
    ops.jpeg_decode(files, chunk_bits=a.chunk)
    torch.cuda.synchronize()
