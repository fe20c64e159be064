#!/bin/bash
set -u
OUT=gpurun_out/r03i
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_wavelet_gpu.py tests/test_pipeline_gpu.py tests/test_configs_gpu.py -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest.txt" 2>&1 || { tail -30 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
bash tools/ab_lib.sh wavelet_bior15 "$OUT/ab" new vf new vf new vf
cp ab/vf.so image-denoising_amd/idn/libidn_hip.so
bash tools/wl_pmc.sh r03i/pmc
