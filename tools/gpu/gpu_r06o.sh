#!/bin/bash
# round 6: synthesis waves-per-EU / rows-per-thread A/B (kernel times)
set -u
bash tools/ab_kern.sh wavelet_haar3 gpurun_out/r06o wl_h3_synth new w4 i4 w4i4 new || exit 1
