#!/bin/bash
# round 5: JPEG GPU tests (arithmetic coding), then the f64 analysis prefetch A/B
set -u
OUT=${1:-r05aa}
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python -u -m pytest tests/test_jpeg_gpu.py tests/test_minibatch_gpu.py -x -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$OUT/pytest.txt 2>&1 \
    || { tail -40 gpurun_out/$OUT/pytest.txt; exit 1; }
tail -1 gpurun_out/$OUT/pytest.txt
cp image-denoising_amd/idn/libidn_hip.so ab/cur.so || exit 1
for op in wavelet_bior15_f64 live_f64; do
  bash tools/ab_lib.sh $op gpurun_out/$OUT/$op old new old new || exit 1
done
cp ab/cur.so image-denoising_amd/idn/libidn_hip.so
