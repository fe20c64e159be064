#!/bin/bash
# round 5: libjpeg 9d block smoothing -- the JPEG GPU tests
set -u
OUT=${1:-r05r}
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python -u -m pytest tests/test_jpeg_gpu.py tests/test_minibatch_gpu.py -x -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/$OUT/pytest.txt 2>&1 || { tail -40 gpurun_out/$OUT/pytest.txt; exit 1; }
tail -1 gpurun_out/$OUT/pytest.txt
