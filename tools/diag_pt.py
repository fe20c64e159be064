"""Diagnose the pitched stencil tile on the GPU (tools only): identity probe (tuning build) and the
three filters against the oracle, printing where mismatches fall."""
import os
import sys

import numpy as np

sys.path.insert(0, "image-denoising_amd")
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import torch  # noqa: E402

import idn  # noqa: E402
import oracle  # noqa: E402
from conftest import textured  # noqa: E402
from idn import _lib  # noqa: E402


def where(got, ref, name):
    bad = np.argwhere(got != ref)
    if len(bad) == 0:
        print(name, "ok")
        return
    print(name, "mismatches", len(bad), "of", got.size)
    for ax, lbl in ((0, "img"), (1, "row"), (2, "col"), (3, "ch")):
        u, c = np.unique(bad[:, ax], return_counts=True)
        print(f"  {lbl}: {len(u)} distinct; first {list(zip(u[:12].tolist(), c[:12].tolist()))}")
    i = tuple(bad[0])
    print("  first", i, "got", got[i], "ref", ref[i])


for shape in [(2, 600, 1000), (1, 13, 664), (2, 7, 104)]:
    img = textured(*shape, seed=7)
    x = torch.from_numpy(img).cuda()
    print("shape", shape)
    os.environ["IDN_STENCIL_IDENT"] = "1"
    with _lib.variant("tuning"):
        y = idn.gaussian_blur(x, 5).cpu().numpy()
    del os.environ["IDN_STENCIL_IDENT"]
    where(y, img, "ident")
    for k in (3, 5):
        where(idn.gaussian_blur(x, k).cpu().numpy(), oracle.cv.gaussian_blur(img, k), f"gauss{k}")
    where(idn.blur(x, 3).cpu().numpy(), oracle.cv.blur(img, 3), "box3")
