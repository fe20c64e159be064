"""Sustained-launch probe: back-to-back launches of one op for a few seconds, timed in blocks
with HIP events on the launch stream; one JSON line per block with the wall time, so the blocks
can be lined up with clock / power samples taken beside it (amd-smi in the calling shell).

    python tools/clock_probe.py --ops gauss5,copy,gauss5 --secs 4 --block 50
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "image-denoising_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="gauss5,copy,box3,gauss5")
    ap.add_argument("--secs", type=float, default=4.0)
    ap.add_argument("--block", type=int, default=50)
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--idle", type=float, default=1.0, help="seconds of idle between ops")
    a = ap.parse_args()
    import torch
    import bench
    import idn
    from idn import ops
    dev = torch.device("cuda:0")
    x = bench.synth_batch(torch, a.n, dev)
    y = torch.empty_like(x)
    nbytes = 2 * x.numel()
    fns = {
        "gauss5": lambda: ops.gaussian_blur(x, 5, out=y),
        "gauss3": lambda: ops.gaussian_blur(x, 3, out=y),
        "box3": lambda: ops.blur(x, 3, out=y),
        "copy": lambda: ops.copy_flat(x, y, 0),
        "copy_nt": lambda: ops.copy_flat(x, y, 1),
    }
    t00 = time.time()
    for spec in a.ops.split(","):
        # "op" or "op:KNOB=v:KNOB2=v" (env knobs the library reads at every launch)
        op, *knobs = spec.split(":")
        for k in list(os.environ):
            if k.startswith("IDN_STENCIL_"):
                del os.environ[k]
        for kv in knobs:
            k, v = kv.split("=")
            os.environ[k] = v
        fn = fns[op]
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        t_end = time.time() + a.secs
        blk = 0
        while time.time() < t_end:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.block):
                fn()
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1) / a.block
            print(json.dumps({"op": spec, "blk": blk, "t": round(time.time() - t00, 3), "abs": round(time.time(), 3),
                              "ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1)}), flush=True)
            blk += 1
        time.sleep(a.idle)


if __name__ == "__main__":
    main()
