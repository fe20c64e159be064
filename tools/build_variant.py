"""Build an A/B variant of the product library with extra compiler flags into ab/<name>.so
(git-ignored; used by tools/ab_lib.sh, which swaps it in on the GPU box).

  python tools/build_variant.py <name> [-DFOO=1 ...]
"""
import concurrent.futures as cf
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "image-denoising_amd"))
from idn import _build  # noqa: E402


def main():
    name, extra = sys.argv[1], sys.argv[2:]
    odir = ROOT / "ab" / ("obj_" + name)
    odir.mkdir(parents=True, exist_ok=True)
    srcs = sorted(_build.CSRC.glob("*.hip"))

    def one(src):
        obj = odir / (src.stem + ".o")
        r = subprocess.run([_build._hipcc(), *_build._flags(), *_build._EXTRA.get(src.name, []), *extra, "-c", str(src), "-o", str(obj)],
                           capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(r.stderr)
        return obj

    with cf.ThreadPoolExecutor(8) as ex:
        objs = list(ex.map(one, srcs))
    out = ROOT / "ab" / (name + ".so")
    subprocess.run([_build._hipcc(), f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-pthread",
                    "-o", str(out), *map(str, objs)], check=True)
    print("built", out)


if __name__ == "__main__":
    main()
