#!/bin/bash
# round 5: JPEG decoder A/B (ab/old.so vs ab/new.so) -- JPEG tests on the new build, then the
# single-file / batch decode times of both builds, interleaved
set -u
OUT=${1:-r05t}
mkdir -p gpurun_out/$OUT
L=image-denoising_amd/idn/libidn_hip.so
cp ab/new.so $L || exit 1
timeout -k 10 600 python -u -m pytest tests/test_jpeg_gpu.py -x -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/$OUT/pytest.txt 2>&1 \
    || { tail -40 gpurun_out/$OUT/pytest.txt; exit 1; }
tail -1 gpurun_out/$OUT/pytest.txt
for v in old new old new; do
  cp ab/$v.so $L || exit 1
  echo "== $v" | tee -a gpurun_out/$OUT/sweep.txt
  timeout -k 10 300 python -u tools/jpeg_chunk_sweep.py --sizes 768,1536,3072 --iters 60 \
      >> gpurun_out/$OUT/sweep.txt 2>&1 || { tail -20 gpurun_out/$OUT/sweep.txt; exit 1; }
done
cp ab/new.so $L
grep -v "^{" gpurun_out/$OUT/sweep.txt | grep -v amdgpu.ids
