#!/bin/bash
# round 6: branch-free counts / slot stores in wl_h3_stats; slot counts and row chunks A/B
set -u
timeout -k 10 300 python -u -m pytest tests/test_wavelet_gpu.py -x -q -k "haar" --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r06i_pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/r06i_pytest.txt; [ $rc = 0 ] || exit $rc
bash tools/ab_kern.sh wavelet_haar3 gpurun_out/r06i wl_h3_stats new k8 k6 it8 new || exit 1
