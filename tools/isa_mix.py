"""Static instruction mix of one kernel in a hipcc --save-temps .s file (tools only).

  python tools/isa_mix.py <file.s> <symbol substring> [--list]
Counts VALU / SALU / LDS / VMEM / branch instructions between the kernel's label and its
.Lfunc_end, and VGPR / SGPR / LDS figures from the kernel descriptor metadata."""
import re
import sys
from collections import Counter


def kernel_body(path, sub):
    lines = open(path).read().splitlines()
    start = None
    for i, l in enumerate(lines):
        head = l.split(" ")[0]
        if start is None and head.endswith(":") and sub in head and head.startswith("_Z"):
            start = i
            name = head[:-1]
        elif start is not None and l.startswith(".Lfunc_end"):
            return name, lines[start + 1:i]
    raise SystemExit(f"no kernel matching {sub}")


def classify(op):
    if op.startswith(("v_",)):
        return "VALU"
    if op.startswith(("s_waitcnt", "s_barrier", "s_nop", "s_endpgm", "s_setprio", "s_sleep")):
        return "sync"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "SMEM"
    if op.startswith("s_"):
        return "SALU"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "VMEM"
    return "other"


def main():
    path, sub = sys.argv[1], sys.argv[2]
    name, body = kernel_body(path, sub)
    c, ops = Counter(), Counter()
    for l in body:
        t = l.strip()
        if not t or t.startswith((";", ".", "_")) or t.endswith(":"):
            continue
        op = t.split()[0]
        c[classify(op)] += 1
        ops[op] += 1
    print(name)
    print(dict(c))
    if "--list" in sys.argv:
        for op, n in ops.most_common():
            print(f"  {n:5d} {op}")


if __name__ == "__main__":
    main()
