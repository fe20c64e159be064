"""Build an A/B variant of the product library with extra compiler flags into ab/<name>.so
(git-ignored; used by tools/ab_lib.sh, which swaps it in on the GPU box).

  python tools/build_variant.py <name> [--base product|tuning] [--only src.hip ...] [-DFOO=1 ...]

--only recompiles just the named sources with the extra flags and links them with the other
sources' objects of the --base build (build/obj or build/obj_tuning; build that first).
"""
import concurrent.futures as cf
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "image-denoising_amd"))
from idn import _build  # noqa: E402


def main():
    name, args = sys.argv[1], sys.argv[2:]
    base, only, extra = "product", [], []
    while args:
        a = args.pop(0)
        if a == "--base":
            base = args.pop(0)
        elif a == "--only":
            only.append(args.pop(0))
        else:
            extra.append(a)
    if base == "tuning":
        extra = ["-DIDN_TUNING_BUILD", *extra]
    odir = ROOT / "ab" / ("obj_" + name)
    odir.mkdir(parents=True, exist_ok=True)
    srcs = sorted(_build.CSRC.glob("*.hip"))
    reuse = []
    if only:
        bdir = _build.TUNING_OBJ_DIR if base == "tuning" else _build.OBJ_DIR
        reuse = [bdir / (s.stem + ".o") for s in srcs if s.name not in only]
        srcs = [s for s in srcs if s.name in only]

    def one(src):
        obj = odir / (src.stem + ".o")
        r = subprocess.run([_build._hipcc(), *_build._flags(), *_build._EXTRA.get(src.name, []), *extra, "-c", str(src), "-o", str(obj)],
                           capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(r.stderr)
        return obj

    with cf.ThreadPoolExecutor(8) as ex:
        objs = list(ex.map(one, srcs)) + reuse
    out = ROOT / "ab" / (name + ".so")
    subprocess.run([_build._hipcc(), f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-pthread",
                    "-o", str(out), *map(str, objs)], check=True)
    print("built", out)


if __name__ == "__main__":
    main()
