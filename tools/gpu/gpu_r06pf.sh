#!/bin/bash
# round 6: the product after the Haar L3 changes -- wavelet / config / jpeg GPU tests, bench lines of
# wavelet_haar3 and cfg5, kernel stats
set -u
OUT=gpurun_out/r06pp
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_wavelet_gpu.py tests/test_configs_gpu.py tests/test_live_path_gpu.py -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $OUT/pytest.txt 2>&1; rc=$?
tail -3 $OUT/pytest.txt; [ $rc = 0 ] || exit $rc
for op in wavelet_haar3 cfg5 wavelet_haar3 cfg5; do
  timeout -k 10 200 python bench.py --op $op --no-cpu --steps 20 --warmup 5 >> $OUT/bench.jsonl 2> $OUT/bench.err || exit 1
  python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1])][-1]; print(d['config']['op'], d['ms_per_step'], d.get('roofline',{}).get('bound'), d.get('roofline',{}).get('frac'))" $OUT/bench.jsonl
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$(pwd)/$OUT/ks" -o k --output-format csv \
  -- python3 bench.py --op wavelet_haar3 --no-cpu --no-copy --steps 10 --warmup 2 > /dev/null 2>&1 || exit 1
