#!/bin/bash
# level-1 synthesis A/B: wl_synth_final3 (product) vs the per-channel streaming kernel (S3=0),
# after the wavelet GPU tests; then kernel stats of the product.  bash tools/wl_s3_ab.sh <out_dir>
set -u
OUT=gpurun_out/${1:-wl_s3_ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 400 python -u -m pytest tests/test_wavelet_gpu.py -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest.txt" 2>&1 || { tail -30 "$OUT/pytest.txt"; exit 1; }
tail -2 "$OUT/pytest.txt"
for rep in 1 2; do
  timeout -k 10 120 python bench.py --op wavelet_bior15 --no-cpu --no-copy >> "$OUT/ab_prod.jsonl" 2>> "$OUT/ab.err" || exit 1
  IDN_WAVELET_S3=0 timeout -k 10 120 python bench.py --op wavelet_bior15 --lib tuning --no-cpu --no-copy >> "$OUT/ab_s3off.jsonl" 2>> "$OUT/ab.err" || exit 1
done
grep -ho '"kernel_ms_avg": [0-9.]*' "$OUT"/ab_*.jsonl
bash tools/ks_op.sh "${1:-wl_s3_ab}/ks" wavelet_bior15
