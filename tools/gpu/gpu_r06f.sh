#!/bin/bash
# round 6: wl_h3_stats occupancy A/B (slots per lane, waves per EU, block rows per workgroup)
set -u
OUT=gpurun_out/r06f
mkdir -p $OUT
for rep in 1 2; do bash tools/ab_lib.sh wavelet_haar3 $OUT/ab$rep k8 wpe1 it8w1 it8 new | grep -v "^ok" || exit 1; done
