#!/bin/bash
# round 5: wavelet f64 analysis prefetch A/B (ab/old.so PF1=1, ab/new.so PF1=5)
set -u
OUT=${1:-r05z}
mkdir -p gpurun_out/$OUT
for op in wavelet_bior15_f64 live_f64; do
  bash tools/ab_lib.sh $op gpurun_out/$OUT/$op old new old new || exit 1
done
