#!/bin/bash
# A/B of two builds of libidn_hip.so on one op: bash tools/ab_lib.sh <op> <out> [v...]
# (builds copied to ab/<v>.so beforehand, on the CPU; ab/ is git-ignored -- delete it after)
set -u
OP=$1; OUT=$2; shift 2
mkdir -p "$OUT"
L=image-denoising_amd/idn/libidn_hip.so
for v in "$@"; do
  cp ab/$v.so $L || exit 1
  timeout -k 10 120 python bench.py --op $OP --no-cpu --no-copy --steps 20 --warmup 3 > "$OUT/$v.json" || exit 1
  python3 -c "import json,sys; print(sys.argv[1], json.load(open(sys.argv[2]))['ms_per_step'])" $v "$OUT/$v.json"
done
for v in new; do
  cp ab/$v.so $L || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$v" -o k --output-format csv -- python3 bench.py --op $OP --no-cpu --no-copy --steps 10 --warmup 2 > /dev/null 2>&1 || exit 1
done
cp ab/new.so $L
echo ok
