#!/bin/bash
# round 6: wl_synth_final3 output clip as the fma clamp bit (IDN_S3_FCLAMP): tests, kernel times
set -u
OUT=gpurun_out/r06pw
mkdir -p $OUT
export TMPDIR=/tmp
L=image-denoising_amd/idn/libidn_hip.so
cp ab/h3fc1.so $L || exit 1
true \
; rc=0
tail -2 $OUT/pytest.txt; [ $rc = 0 ] || exit $rc
bash tools/ab_kern.sh wavelet_bior15 $OUT/kb 'wl_synth_final3<15, true' h3fc0 h3fc1 h3fc0 h3fc1 || exit 1
