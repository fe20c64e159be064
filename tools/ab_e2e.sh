#!/bin/bash
# same-run A/B of libidn_hip.so builds on one op, wall-clock ms_per_step x3 per build, interleaved
#   bash tools/ab_e2e.sh <out_dir> <op> <build> ...   (builds: ab/<build>.so)
set -u
OUT=gpurun_out/$1; OP=$2; shift 2
mkdir -p "$OUT"
L=image-denoising_amd/idn/libidn_hip.so
cp $L ab/_intree.so
for rep in 1 2 3; do
  for v in "$@"; do
    cp ab/$v.so $L || exit 1
    timeout -k 10 120 python bench.py --op $OP --no-cpu --no-copy --steps 20 --warmup 3 >> "$OUT/ab_$v.jsonl" 2>> "$OUT/ab.err" || exit 1
  done
done
cp ab/_intree.so $L
for v in "$@"; do echo "$v $(grep -ho '"ms_per_step": [0-9.]*' "$OUT/ab_$v.jsonl" | tr '\n' ' ')"; done
echo ok
