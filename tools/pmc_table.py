#!/usr/bin/env python3
"""Average the SQ counters of tools/pmc_op.sh runs per variant for kernels matching a substring.
  python tools/pmc_table.py <out_dir> <kernel_substring>"""
import collections
import csv
import glob
import sys

out, ksub = sys.argv[1], sys.argv[2]
for d in sorted(glob.glob(f"{out}/*/")):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"{d}**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if ksub in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(d.rstrip("/").split("/")[-1], {k: f"{sum(v) / len(v):.3e}" for k, v in sorted(agg.items())})
