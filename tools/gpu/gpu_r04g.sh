#!/bin/bash
# round 4: bior1.5 analysis ring loads that really prefetch (unaligned dword per row, refilled after
# the slot's last use, unconditional) -- wavelet tests, A/B against the previous build, kernel
# stats and counter passes of the product.  bash tools/gpu/gpu_r04g.sh
set -u
OUT=gpurun_out/r04g
mkdir -p "$OUT"
export TMPDIR=/tmp
L=image-denoising_amd/idn/libidn_hip.so
cp $L ab/product.so
timeout -k 10 600 python -u -m pytest tests/test_wavelet_gpu.py tests/test_live_path_gpu.py \
    tests/test_pipeline_gpu.py -q --timeout 300 --timeout-method thread -p no:cacheprovider -s \
    > "$OUT/pytest.txt" 2>&1
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
for k in 0 1; do  # integer-key colour stats A/B (tuning build)
  IDN_WAVELET_KEYS=$k timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/ks_keys$k" -o k \
      --output-format csv -- python3 bench.py --op wavelet_haar3 --lib tuning --no-cpu --no-copy \
      --steps 10 --warmup 2 > /dev/null 2>&1 || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/ks_keys$k/k_kernel_stats.csv')):
    if 'color_minmax' in r['Name']: print('keys=$k', r['Name'][:50], round(float(r['AverageNs'])/1e3,1))"
done
bash tools/pmc_r04.sh r04g/pmc wavelet_bior15 || exit 1
python3 - <<'PY'
import csv, glob
for f in glob.glob('gpurun_out/r04g/pmc/wavelet_bior15/ks/**/*kernel_stats.csv', recursive=True):
    for r in list(csv.DictReader(open(f)))[:10]: print(r['Name'][:60], round(float(r['AverageNs'])/1e3, 1))
PY
echo ok
