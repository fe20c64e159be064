#!/bin/bash
# round 5: pitched tile (NB 9), cache bits of the private-row loads and of the stores
set -u
OUT=${1:-r05e}
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python -u -m pytest tests/test_filters_gpu.py -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider -k "pitched or policies or headline" \
    > gpurun_out/$OUT/pytest.txt 2>&1 || { tail -30 gpurun_out/$OUT/pytest.txt; exit 1; }
tail -1 gpurun_out/$OUT/pytest.txt
P=IDN_STENCIL_NTP
bash tools/ab_knobs.sh "$OUT" gauss5 2 "s2:$P=1,IDN_STENCIL_SAUX=2@tnb9" "s16:$P=1,IDN_STENCIL_SAUX=16@tnb9" \
  "s18:$P=1,IDN_STENCIL_SAUX=18@tnb9" "s17:$P=1,IDN_STENCIL_SAUX=17@tnb9" \
  "l16:$P=1,IDN_STENCIL_LAUX=16,IDN_STENCIL_SAUX=2@tnb9" "l18:$P=1,IDN_STENCIL_LAUX=18,IDN_STENCIL_SAUX=2@tnb9" \
  "p4:$P=4,IDN_STENCIL_SAUX=2@tnb9" "nb8s16:$P=1,IDN_STENCIL_SAUX=16@tnb8" || exit 1
