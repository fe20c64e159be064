#!/bin/bash
# round 6: XCD-contiguous order for the Haar-3 statistics / synthesis; tests, kernel times, counters
set -u
timeout -k 10 400 python -u -m pytest tests/test_wavelet_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r06p_pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/r06p_pytest.txt; [ $rc = 0 ] || exit $rc
bash tools/ab_kern.sh wavelet_haar3 gpurun_out/r06p wl_h3 new || exit 1
bash tools/pmc_r04.sh r06p_pmc wavelet_haar3 cfg5 || exit 1
