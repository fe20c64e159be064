"""Build the HIP C-ABI library in-tree: csrc/*.hip -> idn/libidn_hip.so (gfx950 only).

build(tuning=True) builds the tools-only variant idn/libidn_hip_tuning.so (-DIDN_TUNING_BUILD:
the kernels' tuning knobs read from the environment, for A/B runs and the cross-form tests that
load it through idn._lib.variant("tuning")); the product library reads no environment variable.

Driven by ``__graft_entry__.build()`` and by ``python -m idn._build``.  Every translation unit
is compiled with ``hipcc --offload-arch=gfx950 -O3 -ffp-contract=off`` (no FMA contraction:
the noise-apply and blob kernels restate numpy's float64 op order exactly) and linked into
one shared object that ctypes loads (``idn._lib``).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
CSRC = PKG_DIR.parent / "csrc"
LIB_PATH = PKG_DIR / "libidn_hip.so"
TUNING_LIB_PATH = PKG_DIR / "libidn_hip_tuning.so"
OBJ_DIR = PKG_DIR.parent / "build" / "obj"
TUNING_OBJ_DIR = PKG_DIR.parent / "build" / "obj_tuning"
ARCH = "gfx950"


def _hipcc() -> str:
    cand = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not Path(cand).exists():
        raise RuntimeError("hipcc not found; the idn HIP library cannot be built")
    return cand


def _flags() -> list[str]:
    return [
        f"--offload-arch={ARCH}",
        "-O3",
        "-fPIC",
        "-std=c++17",
        "-ffp-contract=off",
        "-fno-gpu-rdc",
        "-Wall",
        "-Wno-unused-function",
        "-Wno-unused-variable",
        f"-I{CSRC}",
    ]


# per-source flags: the two-column bilateral walk (bilateral_u8_pre2_kernel) is one fully unrolled
# loop nest whose pre-unroll body exceeds LLVM's default pragma-unroll size limit; left rolled, its
# shared-weight registers would go to scratch.  The median networks (long runs of independent
# packed min/max) schedule better under LLVM's max-ILP strategy: 5x5 median 0.490 -> 0.479 ms
# (profiles/r04/sched_median_ab.txt; the same strategy made the bilateral and the wavelet slower),
# and so does the k-means fit: quant k=7 2.91 -> 2.84 ms (profiles/r04/sched_ops_ab.txt; noise /
# Poisson / JPEG / stencils: no gain or slower)
_MAX_ILP = ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]
_EXTRA = {"bilateral_u8.hip": ["-mllvm", "-pragma-unroll-threshold=131072"],
          "median_u8.hip": _MAX_ILP, "quant.hip": _MAX_ILP}


def _compile_one(src: Path, tuning: bool = False) -> Path:
    odir = TUNING_OBJ_DIR if tuning else OBJ_DIR
    odir.mkdir(parents=True, exist_ok=True)
    obj = odir / (src.stem + ".o")
    deps = [src] + sorted(CSRC.glob("*.hpp")) + [PKG_DIR.parent.parent / "include" / "idn.h"]
    if obj.exists() and obj.stat().st_mtime >= max(d.stat().st_mtime for d in deps):
        return obj
    cmd = [_hipcc(), *_flags(), *_EXTRA.get(src.name, []),
           *(["-DIDN_TUNING_BUILD"] if tuning else []), "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr}")
    return obj


def build(verbose: bool = False, jobs: int | None = None, tuning: bool = False) -> Path:
    sources = sorted(CSRC.glob("*.hip"))
    if not sources:
        raise RuntimeError(f"no HIP sources under {CSRC}")
    jobs = jobs or min(8, os.cpu_count() or 1, len(sources))
    lib_path = TUNING_LIB_PATH if tuning else LIB_PATH
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile_one(s, tuning), sources))
    newest = max(o.stat().st_mtime for o in objs)
    if not lib_path.exists() or lib_path.stat().st_mtime < newest:
        tmp = lib_path.with_suffix(".so.tmp")
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread", "-o", str(tmp),
               *map(str, objs)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
        os.replace(tmp, lib_path)
    if verbose:
        print(f"built {lib_path}")
    return lib_path


if __name__ == "__main__":
    build(verbose=True)
    build(verbose=True, tuning=True)
    sys.exit(0)
