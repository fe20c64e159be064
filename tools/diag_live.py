"""Diagnostic (tools only): the live test path's bior1.5 denoise at 600x1000 on float64 and u8
input, through several library builds (ab/<name>.so), against the oracle: where the error sits
and how the per-image stats blocks differ.  python tools/diag_live.py old product ..."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "image-denoising_amd", ROOT / "tests"):
    sys.path.insert(0, str(p))

import torch  # noqa: E402
import oracle  # noqa: E402
from conftest import textured  # noqa: E402
from idn import _lib, ops  # noqa: E402


def run(x, name):
    with _lib.variant(name):
        u8, f = ops.denoise_wavelet(x, "bior1.5", None, out="both")
        n, h, w, _ = x.shape
        off = _lib.load().idn_wavelet_stats_offset(n, h, w, ops.WAVELETS["bior1.5"], -1)
    ws = ops._WS_CACHE[(str(x.device), torch.cuda.current_stream(x.device).cuda_stream)]
    st = ws[off:off + n * 256 * 8].view(torch.float64).view(n, 256).cpu().numpy().copy()
    return u8[0].cpu().numpy(), f[0].cpu().numpy().astype(np.float64), st[0]


def main():
    names = sys.argv[1:]
    for nm in names:
        _lib.VARIANTS[nm] = ROOT / "ab" / f"{nm}.so"
    img = textured(1, 600, 1000, seed=2)[0]
    np.random.seed(1234)
    field = np.random.normal(0.0, 0.1 ** 0.5, img.shape)
    noisy = oracle.sk.noise_gaussian(img, field)
    for kind, arr in (("u8", img), ("f64", noisy)):
        ref = oracle.wavelet.denoise_wavelet(arr, "bior1.5", None)
        x = torch.from_numpy(arr[None]).cuda()
        stats = {}
        for nm in names:
            u8, f, st = run(x, nm)
            stats[nm] = st
            err = np.abs(f - ref)
            bad = err > 1e-5
            ys, xs, cs = np.nonzero(bad)
            print(f"{kind} {nm}: max err {err.max():.3g} at {np.unravel_index(err.argmax(), err.shape)}, "
                  f"bad {bad.sum()} ({bad.mean():.3g}); rows {ys.min() if len(ys) else '-'}.."
                  f"{ys.max() if len(ys) else '-'}, cols {xs.min() if len(xs) else '-'}.."
                  f"{xs.max() if len(xs) else '-'}, channels {sorted(set(cs.tolist()))}", flush=True)
            if bad.any():
                rb = np.unique(ys)
                print(f"   bad rows (first 40): {rb[:40].tolist()}  n_rows {len(rb)}")
                cb = np.unique(xs)
                print(f"   bad cols (first 40): {cb[:40].tolist()}  n_cols {len(cb)}")
        L = 3
        for nm in names[1:]:
            a, b = stats[names[0]], stats[nm]
            print(f"  stats {names[0]} vs {nm}: sumsq rel diff "
                  f"{np.abs(a[8:8 + 9 * L] - b[8:8 + 9 * L]).max() / np.abs(a[8:8 + 9 * L]).max():.3g}, "
                  f"medians equal {np.array_equal(a[8 + 9 * L:8 + 9 * L + 3], b[8 + 9 * L:8 + 9 * L + 3])}, "
                  f"thr {a[8 + 9 * L + 3:8 + 9 * L + 3 + 9 * L]} vs {b[8 + 9 * L + 3:8 + 9 * L + 3 + 9 * L]}")


if __name__ == "__main__":
    main()
