#!/bin/bash
# round 6: Haar L3 window sample with IDN_H3_WU items' loads in flight per thread: tests, kernel times
set -u
OUT=gpurun_out/r06pu
mkdir -p $OUT
export TMPDIR=/tmp
L=image-denoising_amd/idn/libidn_hip.so
cp ab/h3wu5.so $L || exit 1
timeout -k 10 400 python -u -m pytest tests/test_wavelet_gpu.py tests/test_configs_gpu.py -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider -k "haar or config5" > $OUT/pytest.txt 2>&1; rc=$?
tail -2 $OUT/pytest.txt; [ $rc = 0 ] || exit $rc
bash tools/ab_kern.sh wavelet_haar3 $OUT/k wl_h3_window h3wu1 h3wu3 h3wu5 h3wu1 h3wu3 h3wu5 || exit 1
