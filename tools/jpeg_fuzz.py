"""Random damaged JPEG files, GPU decode against the oracle (tools only; a robustness sweep
beyond the committed libjpeg-pinned variants): cuts, bit flips, runs of one bits, stray
markers and renumbered restart markers at random places in the small fixtures.
  python tools/jpeg_fuzz.py [--n 300] [--seed 1] [--turbo]"""
import argparse
import random
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "image-denoising_amd"))
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests" / "golden"))

import numpy as np  # noqa: E402

import jpeg_damage as jd  # noqa: E402
from idn import ops  # noqa: E402
from idn._lib import IdnError  # noqa: E402
from oracle import jpeg9  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=300)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--turbo", action="store_true")
    a = ap.parse_args()
    rng = random.Random(a.seed)
    mode = "turbo" if a.turbo else "libjpeg9"
    files = [p for p in sorted((ROOT / "tests/golden/jpeg").glob("*.jpg")) if p.stat().st_size < 20000]
    if a.turbo:
        files = [p for p in files if "smooth" not in p.name and not p.name.startswith("prog")]
    bad = errs = same_err = 0
    t0 = time.time()
    for i in range(a.n):
        p = rng.choice(files)
        data = jd.random_damage(p.read_bytes(), rng)
        try:
            ref = jpeg9.imread(data, mode=mode)
        except Exception as ex:  # the oracle refuses it (e.g. a stray marker it treats as fatal)
            ref = ex
        try:
            got = ops.jpeg_decode([data], mode=mode)[0].cpu().numpy()
        except IdnError as ex:
            got = ex
        if isinstance(ref, Exception) or isinstance(got, Exception):
            if isinstance(ref, Exception) and isinstance(got, Exception):
                same_err += 1
            else:
                errs += 1
                print(f"{i} {p.name}: oracle {type(ref).__name__} / gpu {type(got).__name__}: "
                      f"{ref if isinstance(ref, Exception) else got}", flush=True)
            continue
        if got.shape != ref.shape or not np.array_equal(got, ref):
            bad += 1
            d = np.abs(got.astype(int) - ref.astype(int)) if got.shape == ref.shape else None
            rows = np.nonzero(d.max(axis=(1, 2)))[0] if d is not None else []
            print(f"{i} {p.name}: MISMATCH rows {list(rows[:3])} ({len(rows)})", flush=True)
        if i % 50 == 0:
            print(f"... {i} done, {time.time() - t0:.0f} s", flush=True)
    print(f"fuzz {mode}: {a.n} files, {bad} mismatches, {errs} one-sided errors, "
          f"{same_err} refused by both")


if __name__ == "__main__":
    main()
