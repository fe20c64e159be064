#!/bin/bash
# round 6: block rows per workgroup of the proxy min / max (ITMM 4 / 8 / 16) and of the Haar statistics (IT 8)
set -u
OUT=gpurun_out/r06ps
mkdir -p $OUT
export TMPDIR=/tmp
L=image-denoising_amd/idn/libidn_hip.so
cp ab/h3mm4.so $L || exit 1
timeout -k 10 400 python -u -m pytest tests/test_wavelet_gpu.py -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $OUT/pytest.txt 2>&1; rc=$?
tail -2 $OUT/pytest.txt; [ $rc = 0 ] || exit $rc
bash tools/ab_kern.sh wavelet_bior15 $OUT/kb 'wl_h3_stats<true>' h3mm16 h3mm8 h3mm4 h3mm16 h3mm8 h3mm4 || exit 1
bash tools/ab_kern.sh wavelet_haar3 $OUT/kh 'wl_h3_stats<false>' h3mm4 h3it8 h3mm4 h3it8 || exit 1
