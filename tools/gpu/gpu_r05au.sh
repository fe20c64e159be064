#!/bin/bash
# round 5: checkpoint spacing (JPG_SUB) A/B -- single file and batches, interleaved
set -u
OUT=${1:-r05au}
mkdir -p gpurun_out/$OUT
L=image-denoising_amd/idn/libidn_hip.so
cp $L gpurun_out/$OUT/keep.so
for v in base sub256 sub128 base sub256 sub128; do
  cp ab/$v.so $L || exit 1
  echo "== $v" >> gpurun_out/$OUT/sweep.txt
  timeout -k 10 200 python -u tools/jpeg_chunk_sweep.py --sizes 1536,2560 --iters 40 2>&1 \
      | grep -v "^{" | grep -v amdgpu.ids >> gpurun_out/$OUT/sweep.txt || { cp gpurun_out/$OUT/keep.so $L; exit 1; }
done
cp gpurun_out/$OUT/keep.so $L
rm gpurun_out/$OUT/keep.so
cat gpurun_out/$OUT/sweep.txt
