#!/usr/bin/env python3
"""Tuning sweep for the stripe kernels (run on the GPU box): every combination of the given
environment knobs, interleaved rounds in ONE process, median kernel time via HIP events.  Each
variant's output is compared with the first variant's (the knobs must not change results).

  python tools/sweep_stencil.py --ops gauss5,box3 --env IDN_STENCIL_MAP=0,1,2 --env IDN_BAND_ROWS=0,16,36
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
    ap.add_argument("--env", action="append", default=[], help="NAME=v1,v2,...")
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
        "copy": lambda: y.copy_(x),  # torch's copy kernel on the same buffers (ceiling reference)
    }
    knobs = [(e.split("=")[0], e.split("=")[1].split(",")) for e in args.env]
    names = [k for k, _ in knobs]
    combos = list(itertools.product(*[v for _, v in knobs])) or [()]
    variants = [(op, c) for op in args.ops.split(",") for c in combos]
    res = {v: [] for v in variants}
    ref = {}
    bad = set()
    for rnd in range(args.rounds):
        for v in variants:
            op, c = v
            for k, val in zip(names, c):
                os.environ[k] = val
            fns[op]()
            torch.cuda.synchronize()
            if rnd == 0:
                if op not in ref:
                    ref[op] = y.clone()
                elif not torch.equal(ref[op], y):
                    bad.add(v)
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(args.iters)]
            for a, b in evs:
                a.record()
                fns[op]()
                b.record()
            torch.cuda.synchronize()
            res[v].extend(a.elapsed_time(b) for a, b in evs)
        print(f"round {rnd} done", file=sys.stderr, flush=True)
    nbytes = 6 * args.batch * 600 * 1000
    out = []
    for v, ts in res.items():
        ts.sort()
        med = ts[len(ts) // 2]
        rec = {"op": v[0], **dict(zip(names, v[1])), "ms_median": round(med, 4),
               "ms_min": round(ts[0], 4), "GBps_median": round(nbytes / med / 1e6, 1)}
        if v in bad:
            rec["MISMATCH"] = True
        out.append(rec)
    out.sort(key=lambda r: (r["op"], r["ms_median"]))
    for r in out:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
