#!/bin/bash
# round 5: the scan path's AC refinement staged in LDS, 3-deep bit prefetch, DC refine by OR
set -u
OUT=${1:-r05ak}
mkdir -p gpurun_out/$OUT
timeout -k 10 400 python -u -m pytest tests/test_jpeg_gpu.py tests/test_minibatch_gpu.py -x -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$OUT/pytest.txt 2>&1 \
    || { tail -40 gpurun_out/$OUT/pytest.txt; exit 1; }
tail -1 gpurun_out/$OUT/pytest.txt
timeout -k 10 300 python -u tools/jpeg_paths_time.py --iters 10 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$OUT/paths.txt
