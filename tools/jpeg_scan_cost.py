"""Time per scan of the scan path (tools only): a synthetic 600x1000 q90 progressive file cut after
its k-th scan (EOI appended), decoded for k = 1..all; the differences are the scans' costs.
  python tools/jpeg_scan_cost.py [--iters 5]"""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    x = bench.synth_batch(torch, 1, torch.device("cuda", 0), seed=3).cpu().numpy()
    b = io.BytesIO()
    Image.fromarray(x[0][..., ::-1]).save(b, "JPEG", quality=90, subsampling=2, progressive=True)
    f = b.getvalue()
    sos = [i for i in range(len(f) - 1) if f[i] == 0xFF and f[i + 1] == 0xDA]
    prev = 0.0
    for k in range(1, len(sos) + 1):
        # the scan's header: components, Ss, Se, Ah / Al
        o = sos[k - 1]
        ns = f[o + 4]
        ss, se, a_ = f[o + 5 + 2 * ns], f[o + 6 + 2 * ns], f[o + 7 + 2 * ns]
        end = sos[k] if k < len(sos) else len(f) - 2
        # back up to the marker segments before the next SOS (DHT ...): cut at the first marker
        # after the scan's data
        j = o + 2 + ((f[o + 2] << 8) | f[o + 3])
        while j < end:
            if f[j] == 0xFF and f[j + 1] not in (0x00,) and not 0xD0 <= f[j + 1] <= 0xD7:
                break
            j += 1
        data = f[:j] + b"\xff\xd9"
        ops.jpeg_decode([data])
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.iters):
            t = time.perf_counter()
            ops.jpeg_decode([data])
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t) * 1e3)
        m = statistics.median(ts)
        print(f"scan {k}: comps {ns} Ss {ss} Se {se} Ah {a_ >> 4} Al {a_ & 15}  bytes {j - o:7d}  "
              f"cum {m:8.2f} ms  +{m - prev:7.2f}", flush=True)
        prev = m


if __name__ == "__main__":
    main()
