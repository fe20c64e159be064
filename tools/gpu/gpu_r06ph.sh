#!/bin/bash
# round 6: Haar L3 statistics proxies with one v_min3 / v_max3 per pixel pair (IDN_H3_MIN3): tests, kernel time
set -u
OUT=gpurun_out/r06pi
mkdir -p $OUT
export TMPDIR=/tmp
L=image-denoising_amd/idn/libidn_hip.so
cp ab/h3pk1.so $L || exit 1
timeout -k 10 400 python -u -m pytest tests/test_wavelet_gpu.py tests/test_configs_gpu.py -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider -k "haar or config5" > $OUT/pytest.txt 2>&1; rc=$?
tail -3 $OUT/pytest.txt; [ $rc = 0 ] || exit $rc
bash tools/ab_kern.sh wavelet_haar3 $OUT/k wl_h3_stats h3m1 h3pk1 h3m1 h3pk1
