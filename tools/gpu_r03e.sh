#!/bin/bash
# final3 diagnostics + A/B (wavelet), then the bilateral two-column A/B.
set -u
OUT=gpurun_out/r03e
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_wavelet_gpu.py -k "final3" -q -s --timeout 120 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest_f3.txt" 2>&1
rc=$?
grep -E "final3 vs|passed|failed" "$OUT/pytest_f3.txt"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
for rep in 1 2; do
  timeout -k 10 120 python bench.py --op wavelet_bior15 --no-cpu --no-copy >> "$OUT/wl_prod.jsonl" 2>> "$OUT/ab.err" || exit 1
  IDN_WAVELET_S3=0 timeout -k 10 120 python bench.py --op wavelet_bior15 --lib tuning --no-cpu --no-copy >> "$OUT/wl_s3off.jsonl" 2>> "$OUT/ab.err" || exit 1
done
for f in wl_prod wl_s3off; do echo "$f $(grep -ho '"kernel_ms_avg": [0-9.]*' "$OUT/$f.jsonl" | tr '\n' ' ')"; done
bash tools/bl2_ab.sh r03e/bl2 || exit 1
bash tools/wl_wst_ab.sh r03e/wst
