#!/bin/bash
# round 6: wl_h3_stats kernel-time probes (parts removed: timing only) and moment forms
set -u
bash tools/ab_kern.sh wavelet_haar3 gpurun_out/r06h wl_h3_stats new p1 p2 p4 p8 mom1 new || exit 1
