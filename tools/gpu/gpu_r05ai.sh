#!/bin/bash
# round 5: damaged-file rules with the two-step bad-code length -- JPEG GPU tests, old / new timings
set -u
OUT=${1:-r05ai}
mkdir -p gpurun_out/$OUT
timeout -k 10 400 python -u -m pytest tests/test_jpeg_gpu.py tests/test_minibatch_gpu.py -x -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$OUT/pytest.txt 2>&1 \
    || { tail -40 gpurun_out/$OUT/pytest.txt; exit 1; }
tail -1 gpurun_out/$OUT/pytest.txt
L=image-denoising_amd/idn/libidn_hip.so
cp $L gpurun_out/$OUT/keep.so
for v in old new2 old new2; do
  cp ab/$v.so $L || exit 1
  echo "== $v" >> gpurun_out/$OUT/paths.txt
  timeout -k 10 200 python -u tools/jpeg_paths_time.py --iters 30 2>&1 | grep -v amdgpu.ids >> gpurun_out/$OUT/paths.txt \
      || { cp gpurun_out/$OUT/keep.so $L; exit 1; }
  timeout -k 10 200 python -u tools/jpeg_chunk_sweep.py --sizes 1536,4096 --iters 40 2>&1 \
      | grep -v "^{" | grep -v amdgpu.ids >> gpurun_out/$OUT/paths.txt || true
done
cp gpurun_out/$OUT/keep.so $L
rm gpurun_out/$OUT/keep.so
cat gpurun_out/$OUT/paths.txt
