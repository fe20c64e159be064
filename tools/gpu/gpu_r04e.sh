#!/bin/bash
# round 4: static 5-row sum-of-squares groups in the bior1.5 analysis -- wavelet tests, A/B with
# per-kernel stats of both builds, then the round's counter passes (tools/pmc_r04.sh) and the
# counter list.  bash tools/gpu/gpu_r04e.sh
set -u
OUT=gpurun_out/r04e
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
    timeout -k 10 120 python bench.py --op wavelet_bior15 --no-cpu --no-copy --steps 20 --warmup 3 \
        >> "$OUT/ab_${v}.jsonl" 2>> "$OUT/ab.err" || exit 1
  done
done
for v in old product; do echo "$v $(grep -ho '"kernel_ms_avg": [0-9.]*' "$OUT/ab_${v}.jsonl" | tr '\n' ' ')"; done
for v in old product; do
  cp ab/$v.so $L || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/ks_$v" -o k --output-format csv \
      -- python3 bench.py --op wavelet_bior15 --no-cpu --no-copy --steps 10 --warmup 2 > /dev/null 2>&1 || exit 1
  python3 -c "
import csv
for r in list(csv.DictReader(open('$OUT/ks_$v/k_kernel_stats.csv')))[:9]: print('$v', r['Name'][:60], round(float(r['AverageNs'])/1e3,1))"
done
cp ab/product.so $L
timeout -k 10 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
bash tools/pmc_r04.sh r04e/pmc wavelet_bior15 median5 bilateral gauss5_blob noise_gaussian noise_sap wavelet_haar3 gauss5 || exit 1
echo ok
