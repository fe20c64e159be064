#!/bin/bash
# round 4: exact grid-rounded sums of squares in the bior1.5 analysis -- wavelet tests, then the
# interleaved A/B against round 3's analysis (ab/old) with kernel stats.  bash tools/gpu/gpu_r04d.sh
set -u
OUT=gpurun_out/r04d
mkdir -p "$OUT"
export TMPDIR=/tmp
L=image-denoising_amd/idn/libidn_hip.so
cp $L ab/product.so
timeout -k 10 600 python -u -m pytest tests/test_wavelet_gpu.py tests/test_live_path_gpu.py \
    tests/test_pipeline_gpu.py tests/test_filters_gpu.py -q --timeout 300 --timeout-method thread -p no:cacheprovider -s \
    > "$OUT/pytest.txt" 2>&1
rc=$?
grep -h "LIVE_PATH\|PLAN_FLIPS" "$OUT/pytest.txt" > "$OUT/flips.txt"
tail -3 "$OUT/pytest.txt"
[ $rc = 0 ] || exit $rc
for rep in 1 2; do
  for v in old product g8 g16; do
    cp ab/$v.so $L || exit 1
    for op in wavelet_bior15 wavelet_bior15_f64; do
      timeout -k 10 120 python bench.py --op $op --no-cpu --no-copy --steps 20 --warmup 3 \
          >> "$OUT/ab_${v}_$op.jsonl" 2>> "$OUT/ab.err" || exit 1
    done
  done
done
cp ab/product.so $L
for rep in 1 2; do for pr in 0 1; do
  IDN_MEDIAN_PAIR=$pr timeout -k 10 120 python bench.py --op median5 --lib tuning --no-cpu --no-copy \
      --steps 20 --warmup 3 >> "$OUT/ab_pair_$pr.jsonl" 2>> "$OUT/ab.err" || exit 1
done; done
for pr in 0 1; do echo "pair=$pr median5 $(grep -ho '"kernel_ms_avg": [0-9.]*' "$OUT/ab_pair_$pr.jsonl" | tr '\n' ' ')"; done
for v in old product g8 g16; do for op in wavelet_bior15 wavelet_bior15_f64; do
  echo "$v $op $(grep -ho '"kernel_ms_avg": [0-9.]*' "$OUT/ab_${v}_$op.jsonl" | tr '\n' ' ')"; done; done
cp ab/product.so $L
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/ks_wl" -o k --output-format csv \
    -- python3 bench.py --op wavelet_bior15 --no-cpu --no-copy --steps 10 --warmup 2 > /dev/null 2>&1 || exit 1
python3 -c "
import csv
for r in list(csv.DictReader(open('$OUT/ks_wl/k_kernel_stats.csv')))[:10]: print(r['Name'][:70], round(float(r['AverageNs'])/1e3,1))"
echo ok
