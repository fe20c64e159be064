import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "image-denoising_amd"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built HIP library")


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def textured(n, h, w, c=3, seed=3):
    """BASELINE.md §3 synthetic pattern: clip(128 + 64 sin(2πx/97) cos(2πy/61) + U(-32,32))."""
    import numpy as np
    rs = np.random.RandomState(seed)
    y = np.arange(h)[:, None, None]
    x = np.arange(w)[None, :, None]
    base = 128 + 64 * np.sin(2 * np.pi * x / 97) * np.cos(2 * np.pi * y / 61)
    out = base[None] + rs.uniform(-32, 32, size=(n, h, w, c))
    return np.clip(out, 0, 255).astype(np.uint8)
