#!/bin/bash
# round 5: JPEG Huffman lookup size A/B (ab/old.so = 9 bits, ab/lut11.so, ab/new.so = 12 bits):
# JPEG tests on each, then decode times interleaved
set -u
OUT=${1:-r05y}
mkdir -p gpurun_out/$OUT
L=image-denoising_amd/idn/libidn_hip.so
for v in lut11 new; do
  cp ab/$v.so $L || exit 1
  timeout -k 10 600 python -u -m pytest tests/test_jpeg_gpu.py -x -q --timeout 200 \
      --timeout-method thread -p no:cacheprovider > gpurun_out/$OUT/pytest_$v.txt 2>&1 \
      || { tail -40 gpurun_out/$OUT/pytest_$v.txt; exit 1; }
  echo "$v: $(tail -1 gpurun_out/$OUT/pytest_$v.txt)"
done
for v in old lut11 new old lut11 new; do
  cp ab/$v.so $L || exit 1
  echo "== $v" | tee -a gpurun_out/$OUT/sweep.txt
  timeout -k 10 300 python -u tools/jpeg_chunk_sweep.py --sizes 1536,4096 --iters 60 \
      >> gpurun_out/$OUT/sweep.txt 2>&1 || { tail -20 gpurun_out/$OUT/sweep.txt; exit 1; }
done
cp ab/old.so $L
grep -v "^{" gpurun_out/$OUT/sweep.txt | grep -v amdgpu.ids
