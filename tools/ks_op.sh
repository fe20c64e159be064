#!/bin/bash
# rocprofv3 kernel stats of bench ops: bash tools/ks_op.sh <out_dir> <op> [op ...] (env passes through)
set -u
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
for op in "$@"; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/ks_$op" -o k --output-format csv \
    -- python3 bench.py --op $op --no-cpu --no-copy --steps 20 --warmup 3 > "$OUT/ks_$op.log" 2>&1 || { tail "$OUT/ks_$op.log"; exit 1; }
  python3 - "$OUT/ks_$op/k_kernel_stats.csv" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:8]:
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us {float(r['Percentage']):5.1f}%")
PY
done
