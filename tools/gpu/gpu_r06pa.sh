#!/bin/bash
# round 6: counters of the Haar L3 statistics kernel, product vs the branch-free form (WPE 3)
set -u
L=image-denoising_amd/idn/libidn_hip.so
for v in h3base h3w3; do
  cp ab/$v.so $L || exit 1
  bash tools/pmc_r04.sh r06pa/$v wavelet_haar3 || exit 1
done
cp ab/new.so $L
