"""Dump the wavelet workspace after one GPU call and compare each stage with the oracle."""
import sys
import numpy as np
sys.path.insert(0, "image-denoising_amd"); sys.path.insert(0, "."); sys.path.insert(0, "tests")
import torch, idn
from oracle import wavelet as W
from test_oracle import make_img

shape = tuple(int(v) for v in sys.argv[1:3]) if len(sys.argv) > 2 else (37, 53)
wv = sys.argv[3] if len(sys.argv) > 3 else "bior1.5"
img = make_img(*shape, 8)
h, w = shape
x = torch.from_numpy(img).cuda()
u8, f = idn.ops.denoise_wavelet(x, wv, None, out="both")
torch.cuda.synchronize()
ws = idn.ops._WS_CACHE[str(x.device)].cpu().numpy()
F = len(W.FILTERS[wv][0])
L = max(min(W.dwt_max_level(s, F) for s in shape) - 3, 1)
H1, W1 = (h + F - 1) // 2, (w + F - 1) // 2
fl = ws.view(np.float32)
planes = fl[: 3 * h * w].reshape(3, h, w)
xx = img.astype(np.float64) / 255
Y = xx @ W.YCBCR_FROM_RGB.T + W.YCBCR_OFFSET
print("planes maxdiff", [float(np.abs(planes[c] - Y[..., c]).max()) for c in range(3)])
off = 3 * h * w
bands = fl[off: off + 12 * H1 * W1].reshape(3, 4, H1, W1)
for c in range(3):
    ch = (Y[..., c] - Y[..., c].min()) / (Y[..., c].max() - Y[..., c].min())
    co = W.wavedecn(ch, wv, 1)
    ref = [co[0], co[1]["ad"], co[1]["da"], co[1]["dd"]]
    print("chan", c, "band maxdiff", [float(np.abs(bands[c, b] - ref[b]).max()) for b in range(4)])
# stats
img_floats = (off + 12 * H1 * W1 + 63) // 64 * 64
size_levels = img_floats
st = ws[img_floats * 4: img_floats * 4 + 256 * 8].view(np.float64)
u = st[:3].view(np.uint32).view(np.float32)
print("minmax", u, [(Y[..., c].min(), Y[..., c].max()) for c in range(3)])
for c in range(3):
    ch = (Y[..., c] - Y[..., c].min()) / (Y[..., c].max() - Y[..., c].min())
    co = W.wavedecn(ch, wv, L)
    nz = co[-1]["dd"][np.nonzero(co[-1]["dd"])]
    print("chan", c, "median gpu", st[8 + 9 * L + c], "ref", np.median(np.abs(nz)),
          "sumsq gpu", [st[8 + (c * L + 0) * 3 + b] for b in range(3)],
          "ref", [float((co[-1][k] ** 2).sum()) for k in ("ad", "da", "dd")])
ref = W.denoise_wavelet(img, wv, None)
print("diag counts", st[248:251])
print("final maxdiff", np.abs(f.cpu().numpy() - ref).max())
