#!/bin/bash
# round 6: synthesis with per-thread RGB constants, 2 block rows per thread, 4 waves per SIMD;
# wavelet / config tests, kernel times, haar3 and cfg5 bench lines
set -u
timeout -k 10 400 python -u -m pytest tests/test_wavelet_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r06n_pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/r06n_pytest.txt; [ $rc = 0 ] || exit $rc
bash tools/ab_kern.sh wavelet_haar3 gpurun_out/r06n wl_h3 new || exit 1
bash tools/bench_ops.sh r06n wavelet_haar3 cfg5 || exit 1
