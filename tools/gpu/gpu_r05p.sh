#!/bin/bash
# round 5: table-driven float64 Box-Muller -- noise / live-path tests, then the live path timing
set -u
OUT=${1:-r05p}
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python -u -m pytest tests/test_noise_gpu.py tests/test_live_path_gpu.py \
    tests/test_pipeline_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/$OUT/pytest.txt 2>&1 || { tail -40 gpurun_out/$OUT/pytest.txt; exit 1; }
tail -1 gpurun_out/$OUT/pytest.txt
bash tools/bench_ops.sh "$OUT" live_f64 live_f64_unfused || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$(pwd)/gpurun_out/$OUT/live_prof" -o k \
  --output-format csv -- python3 bench.py --op live_f64 --no-cpu --no-copy --steps 10 --warmup 2 \
  > gpurun_out/$OUT/live_prof.log 2>&1 || exit 1
head -3 gpurun_out/$OUT/live_prof/k_kernel_stats.csv | cut -c1-120
