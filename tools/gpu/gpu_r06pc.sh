#!/bin/bash
# round 6: Haar L3 -- zero counts on the residue branch, level-3 bands across the quad, synthesis
# clip as the packed add's clamp: tests on the new form, kernel times against the product
set -u
OUT=gpurun_out/r06pc
mkdir -p $OUT
L=image-denoising_amd/idn/libidn_hip.so
cp ab/h3v3.so $L || exit 1
timeout -k 10 400 python -u -m pytest tests/test_wavelet_gpu.py tests/test_configs_gpu.py -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider -k "haar or config5" > $OUT/pytest.txt 2>&1; rc=$?
tail -3 $OUT/pytest.txt; [ $rc = 0 ] || exit $rc
bash tools/ab_kern.sh wavelet_haar3 $OUT/k wl_h3_ h3base h3v2 h3v2nc h3v3 h3base h3v2 h3v2nc h3v3
