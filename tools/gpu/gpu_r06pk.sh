#!/bin/bash
# round 6: Haar L3 statistics without the fp64 rescans (timing probe, wrong results) against the product
set -u
bash tools/ab_kern.sh wavelet_haar3 gpurun_out/r06pk/k wl_h3_stats h3prod h3p16 h3prod h3p16 || exit 1
bash tools/ab_kern.sh cfg5 gpurun_out/r06pk/k5 wl_h3_stats h3prod h3p16 || exit 1
