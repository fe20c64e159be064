#!/bin/bash
# round 5: libjpeg's out-of-data rules in every decoder -- old / new interleaved on one box
set -u
OUT=${1:-r05af}
mkdir -p gpurun_out/$OUT
L=image-denoising_amd/idn/libidn_hip.so
cp $L gpurun_out/$OUT/keep.so
for v in old new old new; do
  cp ab/$v.so $L || exit 1
  echo "== $v" >> gpurun_out/$OUT/paths.txt
  timeout -k 10 200 python -u tools/jpeg_paths_time.py --iters 40 >> gpurun_out/$OUT/paths.txt 2>&1 \
      || { tail -20 gpurun_out/$OUT/paths.txt; cp gpurun_out/$OUT/keep.so $L; exit 1; }
  timeout -k 10 200 python -u tools/jpeg_chunk_sweep.py --sizes 1536 --iters 60 2>&1 \
      | grep -v "^{" | grep -v amdgpu.ids >> gpurun_out/$OUT/paths.txt || true
done
cp gpurun_out/$OUT/keep.so $L
rm gpurun_out/$OUT/keep.so
cat gpurun_out/$OUT/paths.txt
