#!/bin/bash
# round 6: integer dot2 colour proxies in wl_h3_stats; wavelet tests, kernel times vs the fp32 proxies
set -u
timeout -k 10 400 python -u -m pytest tests/test_wavelet_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r06m_pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/r06m_pytest.txt; [ $rc = 0 ] || exit $rc
bash tools/ab_kern.sh wavelet_haar3 gpurun_out/r06m wl_h3_s prev new || exit 1
bash tools/ab_kern.sh cfg5 gpurun_out/r06m5 wl_h3_st prev new || exit 1
