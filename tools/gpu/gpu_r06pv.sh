#!/bin/bash
# round 6: Haar L3 window histogram resolution (IDN_H3_MB 6 / 7 / 8 mantissa bits): tests, kernel times, op traffic
set -u
OUT=gpurun_out/r06pv
mkdir -p $OUT
export TMPDIR=/tmp
L=image-denoising_amd/idn/libidn_hip.so
cp ab/h3mb7.so $L || exit 1
timeout -k 10 400 python -u -m pytest tests/test_wavelet_gpu.py tests/test_configs_gpu.py -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider -k "haar or config5" > $OUT/pytest.txt 2>&1; rc=$?
tail -3 $OUT/pytest.txt; [ $rc = 0 ] || exit $rc
cp ab/new.so $L
bash tools/ab_kern.sh wavelet_haar3 $OUT/k wl_h3_ h3mb6 h3mb7 h3mb8 || exit 1
for v in h3mb6 h3mb7 h3mb8; do
  cp ab/$v.so $L || exit 1
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c -d "$(pwd)/$OUT/p_${v}_$c" -o pmc --output-format csv \
      -- python3 bench.py --op wavelet_haar3 --no-cpu --no-copy --steps 3 --warmup 1 --settle-s 0 > $OUT/p_$v.log 2>&1 || exit 1
  done
  python3 - $OUT $v <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(list)
for f in glob.glob(f'{sys.argv[1]}/p_{sys.argv[2]}_*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'wl_h3' in r['Kernel_Name']:
            tot[(r['Kernel_Name'].split('(')[0], r['Counter_Name'])].append(float(r['Counter_Value']))
s = 0
for (k, c), v in sorted(tot.items()):
    b = sum(v) / len(v) * 1024 * (2 if c == 'FETCH_SIZE' else 1)
    s += b
    print(sys.argv[2], k[-22:], c, round(b / 1e6, 1), 'MB')
print(sys.argv[2], 'op total MB', round(s / 1e6, 1), 'x', round(s / 921.6e6, 3))
PY
done
cp ab/new.so $L
