#!/bin/bash
# round 6: bilateral computed colour weights (IDN_BL_CW slot masks) -- accuracy tests and kernel time
set -u
OUT=gpurun_out/r06y
mkdir -p $OUT
export TMPDIR=/tmp
L=image-denoising_amd/idn/libidn_hip.so
for v in cw0 cw1023 cw912 cw960 cw384 cw64; do
  cp ab/$v.so $L || exit 1
  timeout -k 10 300 python -u -m pytest tests/test_filters_gpu.py tests/test_configs_gpu.py -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider -k "bilateral_within_1lsb or config4 or bilateral_shared" \
    > $OUT/pytest_$v.txt 2>&1; rc=$?
  echo "$v tests rc=$rc $(tail -1 $OUT/pytest_$v.txt)"
  [ $rc = 0 ] || [ $rc = 1 ] || exit $rc
done
cp ab/new.so $L
bash tools/ab_kern.sh bilateral $OUT/k bilateral_u8_pre2 cw0 cw1023 cw912 cw960 cw384 cw64 cw0 cw1023
