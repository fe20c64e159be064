#!/bin/bash
# round 6: bior1.5 / other wavelets on u8 input take the Haar path's proxy min / max
# (wl_h3_stats<true>) instead of wl_color_minmax: wavelet + live + config tests, kernel times
set -u
OUT=gpurun_out/r06pr
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_wavelet_gpu.py tests/test_configs_gpu.py tests/test_live_path_gpu.py tests/test_pipeline_gpu.py -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $OUT/pytest.txt 2>&1; rc=$?
tail -3 $OUT/pytest.txt; [ $rc = 0 ] || exit $rc
for op in wavelet_bior15 wavelet_bior15 wavelet_haar3; do
  timeout -k 10 200 python bench.py --op $op --no-cpu --steps 20 --warmup 5 >> $OUT/bench.jsonl 2> $OUT/bench.err || exit 1
  python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1])][-1]; print(d['config']['op'], d['ms_per_step'])" $OUT/bench.jsonl
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$(pwd)/$OUT/ks" -o k --output-format csv \
  -- python3 bench.py --op wavelet_bior15 --no-cpu --no-copy --steps 10 --warmup 2 > /dev/null 2>&1 || exit 1
python3 - $OUT/ks <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + '/*kernel_stats.csv'):
    for r in csv.DictReader(open(f)):
        if 'idn::' in r['Name']: print(r['Name'][:60], round(float(r['AverageNs']) / 1e3, 1))
PY
