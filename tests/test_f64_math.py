"""Accuracy of the table-driven fp64 Box-Muller pieces (csrc/f64_math.hpp) used by the float64
noise stream (noise.hip normal2_f64): tools/check_f64_math.cpp compiles the same header for the
host and compares ln u1, sqrt(-2 ln u1) and (sin, cos)(2 pi u2) with long double over random
53-bit draws plus the edge integers (a + 1 = 1, 2^53; b = 0, 2^53 - 1, the sector boundaries)."""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_table_math_within_two_ulp(tmp_path):
    exe = tmp_path / "check_f64_math"
    subprocess.run(["g++", "-O2", "-std=c++17", f"-I{ROOT / 'image-denoising_amd/csrc'}",
                    str(ROOT / "tools/check_f64_math.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "300000"], check=True, capture_output=True,
                         text=True).stdout
    ln = float(re.search(r"ln u1: worst ([0-9.]+) ulp", out).group(1))
    ln_abs = float(re.search(r"near u1 = 1: ([0-9.e+-]+)", out).group(1))
    rad = float(re.search(r"radius .*: worst ([0-9.]+) ulp", out).group(1))
    m = re.search(r"sin 2 pi u2: worst ([0-9.]+) ulp of 1 .*cos: ([0-9.]+)", out)
    assert ln <= 2.0 and rad <= 2.0, out
    assert ln_abs < 1e-19, out
    assert float(m.group(1)) <= 2.0 and float(m.group(2)) <= 2.0, out
