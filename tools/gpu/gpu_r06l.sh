#!/bin/bash
# round 6: synthesis output stage folded (H3Rgb), fp32 level 1-3, strip grid with a row loop;
# wavelet tests, then synthesis kernel time vs rows per thread
set -u
timeout -k 10 400 python -u -m pytest tests/test_wavelet_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r06l_pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/r06l_pytest.txt; [ $rc = 0 ] || exit $rc
bash tools/ab_kern.sh wavelet_haar3 gpurun_out/r06l wl_h3_synth new s1 s2 s8 new || exit 1
