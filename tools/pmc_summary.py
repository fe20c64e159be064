#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc counter_collection.csv files (host-side helper):

  python tools/pmc_summary.py [--match substr] dir_or_csv ...

prints one line per (kernel, counter) with the mean over dispatches, and for the SQ passes the
derived VALU issue fraction (SQ_ACTIVE_INST_VALU * 4 / SQ_BUSY_CYCLES per SIMD is not used: we
report SQ_INSTS_VALU * 4 cycles / (SQ_BUSY_CYCLES * 4 SIMDs), the guide's issue-rate estimate)
and the LDS bank-conflict share (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE)."""
import argparse
import collections
import csv
from pathlib import Path


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("paths", nargs="+")
    ap.add_argument("--match", default="idn::")
    args = ap.parse_args()
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in args.paths:
        p = Path(p)
        files = ([p] if p.name.endswith(".csv") else []) if p.is_file() else sorted(p.rglob("*counter_collection.csv"))
        for f in files:
            for r in csv.DictReader(open(f)):
                if args.match not in r["Kernel_Name"]:
                    continue
                name = r["Kernel_Name"].split("(")[0].replace("void ", "")
                vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in vals.items():
        print(k)
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        for c in sorted(m):
            print(f"  {c:28s} {m[c]:16.4g}")
        if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE"):
            print(f"  {'lds_conflict_share':28s} {m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']:16.3f}")


if __name__ == "__main__":
    main()
