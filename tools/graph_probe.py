"""Tools only: does replaying the K timed launches as one HIP graph shorten ms_per_step for the
headline 5x5 Gaussian?  Interleaves direct launches and graph replays (steady state), prints the
per-step wall and event times of both.   python tools/graph_probe.py [K] [rounds]"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "image-denoising_amd"))


def main():
    import torch
    import idn
    import bench
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    dev = torch.device("cuda", 0)
    x = bench.synth_batch(torch, 256, dev)
    y = torch.empty_like(x)
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        for _ in range(5):
            idn.gaussian_blur(x, 5, out=y)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(K):
                idn.gaussian_blur(x, 5, out=y)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.5:  # settle, as bench.py
            for _ in range(16):
                idn.gaussian_blur(x, 5, out=y)
            torch.cuda.synchronize()
        res = {"direct": [], "graph": []}
        for _ in range(rounds):
            for form in ("direct", "graph"):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                e0.record(s)
                if form == "graph":
                    g.replay()
                else:
                    for _ in range(K):
                        idn.gaussian_blur(x, 5, out=y)
                e1.record(s)
                torch.cuda.synchronize()
                wall = (time.perf_counter() - t0) / K * 1e3
                res[form].append({"wall_ms": round(wall, 5), "event_ms": round(e0.elapsed_time(e1) / K, 5)})
    ref = y.clone()
    idn.gaussian_blur(x, 5, out=y)
    torch.cuda.synchronize()
    assert torch.equal(ref, y)
    print(json.dumps(res))
    for form, v in res.items():
        w = sorted(r["wall_ms"] for r in v)
        e = sorted(r["event_ms"] for r in v)
        print(form, "wall median", w[len(w) // 2], "event median", e[len(e) // 2],
              "frac(wall)", round(921.6e6 / (w[len(w) // 2] * 1e-3) / 8e12, 4))


if __name__ == "__main__":
    main()
