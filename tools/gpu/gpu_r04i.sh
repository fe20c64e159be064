#!/bin/bash
# round 4: bior1.5 level-1 dd band in fp32 (the sigma median recomputes its exact values from the
# input) -- wavelet tests, A/B against the previous commit's build, and tuning-build kernel stats
# with IDN_WAVELET_DD32=0 / 1 in the same run.  bash tools/gpu/gpu_r04i.sh
set -u
OUT=gpurun_out/r04i
mkdir -p "$OUT"
export TMPDIR=/tmp
L=image-denoising_amd/idn/libidn_hip.so
cp $L ab/product.so
timeout -k 10 600 python -u -m pytest tests/test_wavelet_gpu.py tests/test_live_path_gpu.py \
    tests/test_pipeline_gpu.py tests/test_minibatch_gpu.py -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider -s > "$OUT/pytest.txt" 2>&1
rc=$?
grep -h "LIVE_PATH\|PLAN_FLIPS" "$OUT/pytest.txt" > "$OUT/flips.txt"
tail -2 "$OUT/pytest.txt"
[ $rc = 0 ] || exit $rc
for rep in 1 2; do
  for v in old product; do
    cp ab/$v.so $L || exit 1
    for op in wavelet_bior15 wavelet_bior15_f64; do
      timeout -k 10 120 python bench.py --op $op --no-cpu --no-copy --steps 20 --warmup 3 \
          >> "$OUT/ab_${v}_$op.jsonl" 2>> "$OUT/ab.err" || exit 1
    done
  done
done
for v in old product; do for op in wavelet_bior15 wavelet_bior15_f64; do
  echo "$v $op $(grep -ho '"kernel_ms_avg": [0-9.]*' "$OUT/ab_${v}_$op.jsonl" | tr '\n' ' ')"; done; done
cp ab/product.so $L
for k in 0 1; do
  IDN_WAVELET_DD32=$k timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/ks_dd$k" -o k \
      --output-format csv -- python3 bench.py --op wavelet_bior15 --lib tuning --no-cpu --no-copy \
      --steps 10 --warmup 2 > /dev/null 2>&1 || exit 1
  python3 -c "
import csv
rows = list(csv.DictReader(open('$OUT/ks_dd$k/k_kernel_stats.csv')))
for r in rows[:9]: print('dd32=$k', r['Name'][:58], round(float(r['AverageNs'])/1e3,1))
print('dd32=$k total', round(sum(float(r['TotalDurationNs']) for r in rows if 'idn::' in r['Name'])/10/1e3, 1))"
done
echo ok
