#!/bin/bash
# round 5: SQ counters of the scan path on one progressive 600x1000 file (two passes)
set -u
OUT=gpurun_out/${1:-r05an}
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$(pwd)
i=0
for g in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
         "SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $g -d "$ROOT/$OUT/p$i" -o pmc --output-format csv \
    -- python3 tools/jpeg_single.py --progressive --iters 2 > "$OUT/p$i.log" 2>&1 || { tail "$OUT/p$i.log"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "jpeg_prog_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(acc):
    print(f"{k:24s} {acc[k]:16.0f}")
PY
