#!/bin/bash
# same-run A/B of libidn_hip.so builds on one op: wavelet GPU tests on the product (the in-tree
# library), then kernel_ms_avg x2 per build (interleaved) and per-kernel rocprofv3 stats.
#   bash tools/ab_wavelet.sh <out_dir> <op> <build> ...      (builds: ab/<build>.so; "product" = in-tree)
set -u
OUT=gpurun_out/$1
OP=$2
shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
L=image-denoising_amd/idn/libidn_hip.so
cp $L ab/product.so
timeout -k 10 600 python -u -m pytest tests/test_wavelet_gpu.py tests/test_live_path_gpu.py -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.txt" 2>&1
rc=$?
tail -2 "$OUT/pytest.txt"
[ $rc = 0 ] || exit $rc
for rep in 1 2; do
  for v in "$@"; do
    cp ab/$v.so $L || exit 1
    timeout -k 10 120 python bench.py --op $OP --no-cpu --no-copy --steps 20 --warmup 3 \
        >> "$OUT/ab_$v.jsonl" 2>> "$OUT/ab.err" || exit 1
  done
done
for v in "$@"; do echo "$v $(grep -ho '"kernel_ms_avg": [0-9.]*' "$OUT/ab_$v.jsonl" | tr '\n' ' ')"; done
for v in "$@"; do
  cp ab/$v.so $L || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/ks_$v" -o k --output-format csv \
      -- python3 bench.py --op $OP --no-cpu --no-copy --steps 10 --warmup 2 > /dev/null 2>&1 || exit 1
  python3 -c "
import csv
for r in list(csv.DictReader(open('$OUT/ks_$v/k_kernel_stats.csv')))[:8]: print('$v', r['Name'][:58], round(float(r['AverageNs'])/1e3,1))"
done
cp ab/product.so $L
echo ok
