#!/usr/bin/env python3
"""Fold rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into profiles/pmc_traffic.json.

  python tools/summarize_pmc.py <op> <fetch_dir> <write_dir> <kernel_substring> [algorithmic_bytes]

FETCH_SIZE / WRITE_SIZE are KiB per dispatch.  Per MI355X_MICROARCH.md (HBM section) gfx950's
FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced streaming read, so it is doubled;
WRITE_SIZE is exact for 16 B/lane streaming stores.
"""
import csv
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def avg_counter(d, counter, ksub):
    vals = []
    for f in Path(d).glob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and ksub in r["Kernel_Name"]:
                vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for kernels matching {ksub!r} in {d}")
    return sum(vals) / len(vals), len(vals)


def main():
    op, fdir, wdir, ksub = sys.argv[1:5]
    alg = float(sys.argv[5]) if len(sys.argv) > 5 else None
    fetch_kib, nf = avg_counter(fdir, "FETCH_SIZE", ksub)
    write_kib, nw = avg_counter(wdir, "WRITE_SIZE", ksub)
    read_b = 2.0 * fetch_kib * 1024
    write_b = write_kib * 1024
    out = ROOT / "profiles" / "pmc_traffic.json"
    data = json.loads(out.read_text()) if out.exists() else {}
    data[op] = {
        "kernel": ksub,
        "dispatches": {"fetch": nf, "write": nw},
        "FETCH_SIZE_KiB_raw": round(fetch_kib, 1),
        "WRITE_SIZE_KiB_raw": round(write_kib, 1),
        "hbm_read_bytes_per_launch": int(read_b),
        "hbm_write_bytes_per_launch": int(write_b),
        "hbm_bytes_per_launch": int(read_b + write_b),
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": round((read_b + write_b) / alg, 4) if alg else None,
        "correction": "FETCH_SIZE x2 (gfx950 16B/lane streaming reads), WRITE_SIZE as-is",
    }
    out.write_text(json.dumps(data, indent=1) + "\n")
    print(json.dumps(data[op]))


if __name__ == "__main__":
    main()
