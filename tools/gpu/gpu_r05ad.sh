#!/bin/bash
# round 5: u8 gaussian noise apply by magic-number rounding -- noise GPU tests on the new build,
# then noise_gaussian / cfg2 old vs new
set -u
OUT=${1:-r05ad}
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python -u -m pytest tests/test_noise_gpu.py tests/test_configs_gpu.py \
    tests/test_pipeline_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/$OUT/pytest.txt 2>&1 || { tail -40 gpurun_out/$OUT/pytest.txt; exit 1; }
tail -1 gpurun_out/$OUT/pytest.txt
cp image-denoising_amd/idn/libidn_hip.so ab/cur.so || exit 1
for op in noise_gaussian cfg2; do
  bash tools/ab_lib.sh $op gpurun_out/$OUT/$op old new old new || exit 1
done
cp ab/cur.so image-denoising_amd/idn/libidn_hip.so
