#!/bin/bash
# round 6: fp32 soft thresholds as d - med3(d, -t, t) in the streaming synthesis (IDN_SOFT_MED3): tests, kernel times
set -u
OUT=gpurun_out/r06pt
mkdir -p $OUT
export TMPDIR=/tmp
L=image-denoising_amd/idn/libidn_hip.so
cp ab/h3sm1.so $L || exit 1
timeout -k 10 600 python -u -m pytest tests/test_wavelet_gpu.py tests/test_live_path_gpu.py tests/test_configs_gpu.py -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $OUT/pytest.txt 2>&1; rc=$?
tail -2 $OUT/pytest.txt; [ $rc = 0 ] || exit $rc
bash tools/ab_kern.sh wavelet_bior15 $OUT/kb wl_synth h3sm0 h3sm1 h3sm0 h3sm1 || exit 1
