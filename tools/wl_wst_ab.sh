#!/bin/bash
# streaming-analysis strip width A/B (IDN_WAVELET_WST threads per workgroup, tuning build), after
# the bior1.5 tests under the narrowest strips.  bash tools/wl_wst_ab.sh <out_dir> [widths]
set -u
OUT=gpurun_out/${1:-wl_wst_ab}
W=${2:-"256 128 64"}
mkdir -p "$OUT"
IDN_WAVELET_WST=64 timeout -k 10 300 python -u -m pytest tests/test_wavelet_gpu.py -k "bior15_fp32_analysis" -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.txt" 2>&1 || { tail -30 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
for rep in 1 2; do
  for w in $W; do
    IDN_WAVELET_WST=$w timeout -k 10 120 python bench.py --op wavelet_bior15 --lib tuning --no-cpu --no-copy \
        >> "$OUT/ab_$w.jsonl" 2>> "$OUT/ab.err" || { tail "$OUT/ab.err"; exit 1; }
  done
done
for w in $W; do echo "WST $w $(grep -ho '"kernel_ms_avg": [0-9.]*' "$OUT/ab_$w.jsonl" | tr '\n' ' ')"; done
