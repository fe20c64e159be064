import sys, time, json
sys.path.insert(0, 'image-denoising_amd'); sys.path.insert(0, '.')
import torch, idn
from bench import synth_batch
dev = torch.device('cuda:0')
x = synth_batch(torch, 256, dev); y = torch.empty_like(x)
for _ in range(5): idn.gaussian_blur(x, 5, out=y)
torch.cuda.synchronize()
def run(n, gap_ms=0.0):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record(); idn.gaussian_blur(x, 5, out=y); b.record()
        if gap_ms: torch.cuda.synchronize(); time.sleep(gap_ms/1000)
    torch.cuda.synchronize()
    t = [a.elapsed_time(b) for a, b in ev]
    return t
for label, n, gap in (("burst10", 10, 0), ("burst50", 50, 0), ("burst200", 200, 0), ("gap1ms x20", 20, 1.0), ("gap20ms x20", 20, 20.0), ("burst400", 400, 0)):
    t = run(n, gap)
    q = sorted(t)
    print(label, "first5", [round(v,4) for v in t[:5]], "last5", [round(v,4) for v in t[-5:]], "median", round(q[len(q)//2],4), "min", round(q[0],4), flush=True)
