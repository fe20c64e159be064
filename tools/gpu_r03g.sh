#!/bin/bash
# wavelet (superstep analysis) + bilateral tests, Gaussian LDS-DMA A/B, wavelet library A/B.
set -u
OUT=gpurun_out/r03g
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_wavelet_gpu.py tests/test_filters_gpu.py -k "not lds_dma" -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest.txt" 2>&1 || { tail -30 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
for rep in 1 2 3; do
  timeout -k 10 120 python bench.py --op gauss5 --no-cpu --no-copy >> "$OUT/g5.jsonl" 2>> "$OUT/ab.err" || exit 1
  IDN_STENCIL_GLDS=1 timeout -k 10 120 python bench.py --op gauss5 --lib tuning --no-cpu --no-copy >> "$OUT/g5glds.jsonl" 2>> "$OUT/ab.err" || exit 1
done
for f in g5 g5glds; do echo "$f $(grep -ho '"frac": [0-9.]*' "$OUT/$f.jsonl" | tr '\n' ' ')"; done
timeout -k 10 120 python -u -m pytest tests/test_filters_gpu.py -k "lds_dma" -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest_glds.txt" 2>&1; tail -1 "$OUT/pytest_glds.txt"
bash tools/ab_lib.sh wavelet_bior15 "$OUT/wl" new ss2 wlm512 wlm1024 new ss2 wlm512 wlm1024; cp ab/new.so ab/old.so
