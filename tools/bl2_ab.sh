#!/bin/bash
# bilateral two-column kernel (product) vs the one-column kernel (IDN_BL2=0), after the bilateral
# GPU tests.   bash tools/bl2_ab.sh <out_dir>
set -u
OUT=gpurun_out/${1:-bl2_ab}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_filters_gpu.py tests/test_configs_gpu.py -k "bilateral or config4" -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.txt" 2>&1 || { tail -30 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
for rep in 1 2; do
  timeout -k 10 120 python bench.py --op bilateral --no-cpu --no-copy >> "$OUT/ab_prod.jsonl" 2>> "$OUT/ab.err" || exit 1
  IDN_BL2=0 timeout -k 10 120 python bench.py --op bilateral --lib tuning --no-cpu --no-copy >> "$OUT/ab_bl1.jsonl" 2>> "$OUT/ab.err" || exit 1
  IDN_BL2_WG=3 timeout -k 10 120 python bench.py --op bilateral --lib tuning --no-cpu --no-copy >> "$OUT/ab_wg3.jsonl" 2>> "$OUT/ab.err" || exit 1
done
for f in prod bl1 wg3; do echo "$f $(grep -ho '"kernel_ms_avg": [0-9.]*' "$OUT/ab_$f.jsonl" | tr '\n' ' ')"; done
