#!/usr/bin/env python3
"""VALU issue roofline of a kernel from a tools/pmc_valu.sh pass and its rocprofv3 kernel time.

  python tools/valu_roofline.py <pmc_dir_of_op> <kernel_substring> <kernel_ms>

utilisation = SQ_INSTS_VALU (wave-instructions, whole chip, per dispatch) x 4 cycles (a wave64
VALU instruction on a 16-lane SIMD) / (kernel time x 2.4 GHz x 1024 SIMDs).  The clock is the
nominal one: under load the chip runs slower (MI355X_MICROARCH.md, DVFS), so this is a lower
bound of the true issue utilisation.  LDS: SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE."""
import collections
import csv
import glob
import json
import sys

d, ksub, ms = sys.argv[1], sys.argv[2], float(sys.argv[3])
agg = collections.defaultdict(list)
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if ksub in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
avg = {k: sum(v) / len(v) for k, v in agg.items()}
util = avg["SQ_INSTS_VALU"] * 4 / (ms * 1e-3 * 2.4e9 * 1024)
lds = avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_LDS_IDX_ACTIVE"] if avg.get("SQ_LDS_IDX_ACTIVE") else 0.0
print(json.dumps({"kernel": ksub, "kernel_ms": ms, "valu_wave_instr": avg["SQ_INSTS_VALU"],
                  "valu_issue_util": round(util, 3), "lds_wave_instr": avg.get("SQ_INSTS_LDS", 0.0),
                  "lds_conflict_share": round(lds, 3)}))
