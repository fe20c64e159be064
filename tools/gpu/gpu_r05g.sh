#!/bin/bash
# round 5: fused blob epilogue on the pitched tile, the round's test fixes (jpeg, wavelet), then
# blob band height x policy
set -u
OUT=${1:-r05g}
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_jpeg_gpu.py \
    tests/test_live_path_gpu.py tests/test_wavelet_gpu.py -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/$OUT/pytest.txt 2>&1 \
    || { tail -30 gpurun_out/$OUT/pytest.txt; exit 1; }
tail -1 gpurun_out/$OUT/pytest.txt
bash tools/ab_knobs.sh "$OUT" gauss5_blob 2 product "flat:IDN_STENCIL_FORM=0" \
  "nb9d:IDN_STENCIL_NTP=0,IDN_STENCIL_NTS=0" "nb9st:IDN_STENCIL_NTP=0" \
  "nb6:X=0@tbl6" "nb6d:IDN_STENCIL_NTP=0,IDN_STENCIL_NTS=0@tbl6" "nb8:X=0@tbl8" || exit 1
