#!/bin/bash
# round 6: Haar L3 statistics timing probes (wrong results by design: kernel time only) and the
# counters of the product vs the branch-free form
set -u
bash tools/ab_kern.sh wavelet_haar3 gpurun_out/r06pb/k wl_h3_stats h3base h3w3 h3p32 h3p64 h3p66 h3p1 h3p8 h3p4 h3base h3w3 || exit 1
L=image-denoising_amd/idn/libidn_hip.so
for v in h3base h3w3; do
  cp ab/$v.so $L || exit 1
  bash tools/pmc_r04.sh r06pb/$v wavelet_haar3 || exit 1
done
cp ab/new.so $L
