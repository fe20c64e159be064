#!/usr/bin/env python3
"""Tuning sweep for the stencil kernels (run on the GPU box): interleaved rounds of each
(op, IDN_BAND_ROWS, IDN_STENCIL_NT) variant in ONE process, median kernel time via HIP events.

  python tools/sweep_stencil.py [--batch 256] [--rounds 5] [--ops gauss5,box3]
"""
import argparse
import itertools
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "image-denoising_amd"))
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--ops", default="gauss5")
    ap.add_argument("--bands", default="0,60,100,150,300")
    ap.add_argument("--nt", default="0,1,2,3")
    args = ap.parse_args()
    import torch
    import idn
    from bench import synth_batch
    dev = torch.device("cuda:0")
    x = synth_batch(torch, args.batch, dev)
    y = torch.empty_like(x)
    fns = {
        "gauss5": lambda: idn.gaussian_blur(x, 5, out=y),
        "gauss3": lambda: idn.gaussian_blur(x, 3, out=y),
        "box3": lambda: idn.blur(x, 3, out=y),
        "median3": lambda: idn.median_blur(x, 3, out=y),
        "median5": lambda: idn.median_blur(x, 5, out=y),
        "bilateral": lambda: idn.bilateral_filter(x, 9, 75.0, 75.0, out=y),
    }
    variants = list(itertools.product(args.ops.split(","), args.bands.split(","), args.nt.split(",")))
    res = {v: [] for v in variants}
    for _ in range(args.rounds):
        for v in variants:
            op, br, nt = v
            os.environ["IDN_BAND_ROWS"] = br
            os.environ["IDN_STENCIL_NT"] = nt
            fns[op]()
            torch.cuda.synchronize()
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(args.iters)]
            for a, b in evs:
                a.record()
                fns[op]()
                b.record()
            torch.cuda.synchronize()
            res[v].extend(a.elapsed_time(b) for a, b in evs)
    nbytes = 6 * args.batch * 600 * 1000
    out = []
    for v, ts in res.items():
        ts.sort()
        med = ts[len(ts) // 2]
        out.append({"op": v[0], "band_rows": v[1], "nt": v[2], "ms_median": round(med, 4),
                    "ms_min": round(ts[0], 4), "GBps_median": round(nbytes / med / 1e6, 1)})
    out.sort(key=lambda r: (r["op"], r["ms_median"]))
    for r in out:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
