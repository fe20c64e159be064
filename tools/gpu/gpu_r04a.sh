#!/bin/bash
# round 4, first GPU call: the whole -m gpu suite (live-path + batch-invariance tests, flip shares
# printed), then an interleaved A/B of the bior1.5 op over three builds (ab/old = round 3's
# analysis, ab/wpe1 / ab/wpe6 = per-group sums of squares without / with the 6-wave bound for the
# fp32 deeper levels) with kernel stats per build.  bash tools/gpu/gpu_r04a.sh
set -u
OUT=gpurun_out/r04a
mkdir -p "$OUT"
export TMPDIR=/tmp
L=image-denoising_amd/idn/libidn_hip.so
cp $L ab/product.so
timeout -k 10 200 python -u tools/diag_live.py old wpe1 product > "$OUT/diag.txt" 2>&1 || exit 1
grep -v "^ " "$OUT/diag.txt" | cut -c1-200
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider -s > "$OUT/pytest.txt" 2>&1
rc=$?
grep -h "LIVE_PATH\|PLAN_FLIPS" "$OUT/pytest.txt" > "$OUT/flips.txt"
tail -4 "$OUT/pytest.txt"
[ $rc = 0 ] || exit $rc
for rep in 1 2; do
  for v in old wpe1 wpe6; do
    cp ab/$v.so $L || exit 1
    for op in wavelet_bior15 wavelet_bior15_f64; do
      timeout -k 10 120 python bench.py --op $op --no-cpu --no-copy --steps 20 --warmup 3 \
          >> "$OUT/ab_${v}_$op.jsonl" 2>> "$OUT/ab.err" || exit 1
    done
  done
done
for v in old wpe1 wpe6; do
  for op in wavelet_bior15 wavelet_bior15_f64; do
    echo "$v $op $(grep -ho '"kernel_ms_avg": [0-9.]*' "$OUT/ab_${v}_$op.jsonl" | tr '\n' ' ')"
  done
done
for v in old wpe1 wpe6; do
  cp ab/$v.so $L || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/ks_$v" -o k --output-format csv \
      -- python3 bench.py --op wavelet_bior15 --no-cpu --no-copy --steps 10 --warmup 2 > /dev/null 2>&1 || exit 1
done
cp ab/product.so $L
echo ok
