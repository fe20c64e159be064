#!/bin/bash
# deeper-level synthesis A/B: wl_synth_final3<FM, false> at levels >= 2 with output width >= W
# (IDN_WAVELET_S3D=W, tuning build) vs the streaming kernel (tuning default), after the deeper
# bitwise test; then kernel stats of the all-levels form.  bash tools/wl_s3d_ab.sh <out_dir>
set -u
OUT=gpurun_out/${1:-wl_s3d_ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_wavelet_gpu.py -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider -k "final3" -s > "$OUT/pytest.txt" 2>&1 || { tail -30 "$OUT/pytest.txt"; exit 1; }
grep -h "differ\|passed" "$OUT/pytest.txt" | sort | uniq -c
for rep in 1 2; do
  for w in 1073741824 0 384 200; do
    IDN_WAVELET_S3D=$w timeout -k 10 120 python bench.py --op wavelet_bior15 --lib tuning --no-cpu --no-copy >> "$OUT/ab_$w.jsonl" 2>> "$OUT/ab.err" || exit 1
  done
done
for w in 1073741824 0 384 200; do echo "S3D $w $(grep -ho '"kernel_ms_avg": [0-9.]*' "$OUT/ab_$w.jsonl" | tr '\n' ' ')"; done
IDN_WAVELET_S3D=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/ks" -o k --output-format csv -- python3 bench.py --op wavelet_bior15 --lib tuning --no-cpu --no-copy --steps 10 --warmup 2 > /dev/null 2>&1 || exit 1
cut -c1-150 "$OUT"/ks/k_kernel_stats.csv | head -12
