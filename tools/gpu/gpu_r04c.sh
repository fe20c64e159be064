#!/bin/bash
# round 4: wavelet per-thread group partials + 24-byte-lane 5x5 median.  Tests of both, then
# interleaved A/Bs: bior1.5 op (ab/old = round 3's analysis vs the product), median5 op and
# config 3 (tuning build: IDN_MEDIAN_W24=0 vs 1), kernel stats.  bash tools/gpu/gpu_r04c.sh
set -u
OUT=gpurun_out/r04c
mkdir -p "$OUT"
export TMPDIR=/tmp
L=image-denoising_amd/idn/libidn_hip.so
cp $L ab/product.so
timeout -k 10 600 python -u -m pytest tests/test_wavelet_gpu.py tests/test_live_path_gpu.py \
    tests/test_filters_gpu.py tests/test_pipeline_gpu.py tests/test_configs_gpu.py -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider -s > "$OUT/pytest.txt" 2>&1
rc=$?
grep -h "LIVE_PATH\|PLAN_FLIPS" "$OUT/pytest.txt" > "$OUT/flips.txt"
tail -4 "$OUT/pytest.txt"
[ $rc = 0 ] || exit $rc
for rep in 1 2; do
  for v in old product; do
    cp ab/$v.so $L || exit 1
    timeout -k 10 120 python bench.py --op wavelet_bior15 --no-cpu --no-copy --steps 20 --warmup 3 \
        >> "$OUT/ab_${v}_wl.jsonl" 2>> "$OUT/ab.err" || exit 1
  done
  cp ab/product.so $L
  for w in 0 1; do
    for op in median5 cfg3; do
      IDN_MEDIAN_W24=$w timeout -k 10 120 python bench.py --op $op --lib tuning --no-cpu --no-copy \
          --steps 20 --warmup 3 >> "$OUT/ab_w24_${w}_$op.jsonl" 2>> "$OUT/ab.err" || exit 1
    done
  done
done
for v in old product; do echo "$v wl $(grep -ho '"kernel_ms_avg": [0-9.]*' "$OUT/ab_${v}_wl.jsonl" | tr '\n' ' ')"; done
for w in 0 1; do for op in median5 cfg3; do echo "w24=$w $op $(grep -ho '"kernel_ms_avg": [0-9.]*' "$OUT/ab_w24_${w}_$op.jsonl" | tr '\n' ' ')"; done; done
cp ab/product.so $L
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/ks_wl" -o k --output-format csv \
    -- python3 bench.py --op wavelet_bior15 --no-cpu --no-copy --steps 10 --warmup 2 > /dev/null 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/ks_med" -o k --output-format csv \
    -- python3 bench.py --op median5 --no-cpu --no-copy --steps 10 --warmup 2 > /dev/null 2>&1 || exit 1
echo ok
