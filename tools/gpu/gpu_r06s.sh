#!/bin/bash
# round 6: window-relative sigma select; stats rows-per-workgroup A/B; tests + bench lines
set -u
timeout -k 10 400 python -u -m pytest tests/test_wavelet_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r06s_pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/r06s_pytest.txt; [ $rc = 0 ] || exit $rc
bash tools/ab_kern.sh wavelet_haar3 gpurun_out/r06s wl_h3_s new it8 new || exit 1
bash tools/bench_ops.sh r06s wavelet_haar3 cfg5 || exit 1
