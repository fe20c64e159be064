#!/bin/bash
# round 6: bior1.5 level-1 analysis in fp32 with integer-key codes (A32=7) vs the fp64 highpass
# (A32=3): wavelet tests, kernel times of both forms (tuning build)
set -u
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_wavelet_gpu.py -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r06t_pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/r06t_pytest.txt; [ $rc = 0 ] || exit $rc
for v in 3 7; do
  IDN_WAVELET_A32=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$(pwd)/gpurun_out/r06t/a$v" -o k --output-format csv \
    -- python3 bench.py --lib tuning --op wavelet_bior15 --no-cpu --no-copy --steps 10 --warmup 2 > gpurun_out/r06t_a$v.log 2>&1 || exit 1
  python3 - gpurun_out/r06t/a$v $v <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + '/*kernel_stats.csv'):
    for r in csv.DictReader(open(f)):
        if 'idn' in r['Name']: print(sys.argv[2], r['Name'][:50], round(float(r['AverageNs']) / 1e3, 1))
PY
done
