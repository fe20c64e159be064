#!/bin/bash
# kernel times of one op under several builds: bash tools/ab_kern.sh <op> <out> <kernel-substr> v...
# (builds in ab/<v>.so, swapped in for each run; ab/new.so restored at the end)
set -u
OP=$1; OUT=$2; KS=$3; shift 3
mkdir -p "$OUT"
L=image-denoising_amd/idn/libidn_hip.so
export TMPDIR=/tmp
for v in "$@"; do
  cp ab/$v.so $L || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$(pwd)/$OUT/$v" -o k --output-format csv \
    -- python3 bench.py --op $OP --no-cpu --no-copy --steps 10 --warmup 2 > /dev/null 2>&1 || exit 1
  python3 - "$OUT/$v" "$KS" "$v" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + '/*kernel_stats.csv'):
    for r in csv.DictReader(open(f)):
        if sys.argv[2] in r['Name']:
            print(sys.argv[3], r['Name'][:40], round(float(r['AverageNs']) / 1e3, 1))
PY
done
cp ab/new.so $L
