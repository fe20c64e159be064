#!/bin/bash
# SQ instruction-mix pass (tools/pmc_op.sh counters) over the VALU-bound ops, one pass per op.
#   bash tools/pmc_valu.sh <out_dir>
set -u
OUT=$1
for op in median5 bilateral noise_gaussian wavelet_haar3 gauss5; do
  bash tools/pmc_op.sh $op "$OUT/$op" || exit 1
done
echo ok
