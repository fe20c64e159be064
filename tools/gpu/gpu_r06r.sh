#!/bin/bash
# round 6: rescan only the masked steps; synthesis XCD order A/B; tests, kernel times, FETCH
set -u
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_wavelet_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r06r_pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/r06r_pytest.txt; [ $rc = 0 ] || exit $rc
bash tools/ab_kern.sh wavelet_haar3 gpurun_out/r06r wl_h3_s new sx new || exit 1
L=image-denoising_amd/idn/libidn_hip.so
for v in new p16; do
  cp ab/$v.so $L
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d "$(pwd)/gpurun_out/r06r/f_$v" -o pmc --output-format csv \
    -- python3 bench.py --op wavelet_haar3 --no-cpu --no-copy --steps 3 --warmup 1 --settle-s 0 > /dev/null 2>&1 || exit 1
  python3 - gpurun_out/r06r/f_$v $v <<'PY'
import csv, glob, sys, collections
v = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + '/*counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        if 'h3_stats' in r['Kernel_Name']: v[r['Counter_Name']].append(float(r['Counter_Value']))
print(sys.argv[2], {k: round(sum(x) / len(x) * 1024 / 1e6, 1) for k, x in v.items()})
PY
done
cp ab/new.so $L
