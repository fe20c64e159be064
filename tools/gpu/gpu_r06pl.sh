#!/bin/bash
# round 6: Haar L3 rescans with IDN_H3_RB steps' loads in flight: tests on RB=4, kernel times
set -u
OUT=gpurun_out/r06po
mkdir -p $OUT
export TMPDIR=/tmp
L=image-denoising_amd/idn/libidn_hip.so
cp ab/h3spk1.so $L || exit 1
timeout -k 10 400 python -u -m pytest tests/test_wavelet_gpu.py tests/test_configs_gpu.py -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider -k "haar or config5" > $OUT/pytest.txt 2>&1; rc=$?
tail -3 $OUT/pytest.txt; [ $rc = 0 ] || exit $rc
cp ab/new.so $L
bash tools/ab_kern.sh wavelet_haar3 $OUT/k wl_h3_synth h3prod h3spk1 h3prod h3spk1 || exit 1
bash tools/ab_kern.sh cfg5 $OUT/k5 wl_h3_synth h3prod h3spk1 || exit 1
