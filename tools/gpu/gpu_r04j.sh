#!/bin/bash
# round 4: A/B of the level-1 analysis row-task spread (IDN_WS_SPREAD=1 build: every wave of the
# workgroup takes a contiguous run of row tasks) against the product, same run; wavelet tests on
# the variant.  bash tools/gpu/gpu_r04j.sh
set -u
OUT=gpurun_out/r04j
mkdir -p "$OUT"
export TMPDIR=/tmp
L=image-denoising_amd/idn/libidn_hip.so
cp $L ab/product.so
cp ab/spread.so $L
timeout -k 10 600 python -u -m pytest tests/test_wavelet_gpu.py tests/test_live_path_gpu.py -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.txt" 2>&1
rc=$?
cp ab/product.so $L
tail -2 "$OUT/pytest.txt"
[ $rc = 0 ] || exit $rc
VS="product spread"
for rep in 1 2; do
  for v in $VS; do
    cp ab/$v.so $L || exit 1
    timeout -k 10 120 python bench.py --op wavelet_bior15 --no-cpu --no-copy --steps 20 --warmup 3 \
        >> "$OUT/ab_$v.jsonl" 2>> "$OUT/ab.err" || exit 1
  done
done
for v in $VS; do echo "$v $(grep -ho '"kernel_ms_avg": [0-9.]*' "$OUT/ab_$v.jsonl" | tr '\n' ' ')"; done
for v in $VS; do
  cp ab/$v.so $L || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/ks_$v" -o k --output-format csv \
      -- python3 bench.py --op wavelet_bior15 --no-cpu --no-copy --steps 10 --warmup 2 > /dev/null 2>&1 || exit 1
  python3 -c "
import csv
for r in list(csv.DictReader(open('$OUT/ks_$v/k_kernel_stats.csv')))[:5]: print('$v', r['Name'][:58], round(float(r['AverageNs'])/1e3,1))"
done
cp ab/product.so $L
echo ok
