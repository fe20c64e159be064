#!/bin/bash
# round 5: pitched tile, waves per segment x band height (split policy), parity first
set -u
OUT=${1:-r05d}
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python -u -m pytest tests/test_filters_gpu.py -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider -k "pitched or policies" \
    > gpurun_out/$OUT/pytest.txt 2>&1 || { tail -30 gpurun_out/$OUT/pytest.txt; exit 1; }
tail -1 gpurun_out/$OUT/pytest.txt
S="IDN_STENCIL_NTP=1,IDN_STENCIL_NTS=1"
bash tools/ab_knobs.sh "$OUT" gauss5 2 "nb9s:$S@tnb9" "nb8s:$S@tnb8" "nb8w2:$S,IDN_STENCIL_WPS=2@tnb8" \
  "nb10s:$S@tnb10" "nb10w2:$S,IDN_STENCIL_WPS=2@tnb10" "nb12w2:$S,IDN_STENCIL_WPS=2@tnb12" \
  "nb6w2:$S,IDN_STENCIL_WPS=2" || exit 1
