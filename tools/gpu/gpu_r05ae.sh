#!/bin/bash
# round 5: early-exit B passes (12 per host round trip) -- JPEG tests, decode times, a trace
set -u
OUT=${1:-r05ae}
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python -u -m pytest tests/test_jpeg_gpu.py tests/test_minibatch_gpu.py -x -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$OUT/pytest.txt 2>&1 \
    || { tail -40 gpurun_out/$OUT/pytest.txt; exit 1; }
tail -1 gpurun_out/$OUT/pytest.txt
timeout -k 10 300 python -u tools/jpeg_chunk_sweep.py --sizes 1536,4096 --iters 60 \
    > gpurun_out/$OUT/sweep.txt 2>&1 || { tail -20 gpurun_out/$OUT/sweep.txt; exit 1; }
grep -v "^{" gpurun_out/$OUT/sweep.txt | grep -v amdgpu.ids
timeout -k 10 300 rocprofv3 --kernel-trace -d "$(pwd)/gpurun_out/$OUT/tr" -o k --output-format csv \
    -- python3 tools/jpeg_single.py --iters 20 > gpurun_out/$OUT/tr.log 2>&1 || exit 1
python3 tools/timeline.py gpurun_out/$OUT/tr/k_kernel_trace.csv jpeg_unstuff_count 3 \
    > gpurun_out/$OUT/timeline.txt || exit 1
tail -1 gpurun_out/$OUT/timeline.txt
