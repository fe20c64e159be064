"""JPEG decode time vs the entropy chunk size (tools only): one 600x1000 q90 4:2:0 file and a
batch of 256, each chunk size timed over many synchronous calls (median of per-call wall times).
  python tools/jpeg_chunk_sweep.py [--sizes 1024,2048,4096] [--iters 100]"""
import argparse
import io
import json
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1024,1536,2048,3072,4096")
    ap.add_argument("--iters", type=int, default=100)
    args = ap.parse_args()
    x = bench.synth_batch(torch, 256, torch.device("cuda", 0), seed=3).cpu().numpy()
    files = []
    for im in x:
        b = io.BytesIO()
        Image.fromarray(im[..., ::-1]).save(b, "JPEG", quality=90, subsampling=2)
        files.append(b.getvalue())
    ref1 = ops.jpeg_decode(files[:1])
    refn = ops.jpeg_decode(files)
    out = {}
    for cb in [int(s) for s in args.sizes.split(",")]:
        for name, fl, ref, iters in (("single", files[:1], ref1, args.iters),
                                     ("batch256", files, refn, max(10, args.iters // 10))):
            y = ops.jpeg_decode(fl, chunk_bits=cb)
            assert torch.equal(y, ref), (cb, name)
            ts = []
            for _ in range(iters):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                ops.jpeg_decode(fl, chunk_bits=cb)
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t0) * 1e3)
            out[f"{name}@{cb}"] = round(statistics.median(ts), 4)
            print(name, cb, out[f"{name}@{cb}"], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
