#!/bin/bash
# round 6: Haar L3 statistics -- zero counts (ZC) x level-3 bands across the quad (L3Q), kernel times
set -u
bash tools/ab_kern.sh wavelet_haar3 gpurun_out/r06pe/k wl_h3_stats h3base h3s01 h3b001 h3b011 h3b000 h3b001w1 h3base h3s01 h3b001 h3b011 h3b000 h3b001w1
