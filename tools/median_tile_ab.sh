#!/bin/bash
# median LDS band-tile vs stripe form: parity tests (both forms forced), then bench lines
set -u
mkdir -p gpurun_out/mta
for t in 1 0; do
  IDN_MEDIAN_TILE=$t timeout -k 10 200 python -u -m pytest tests/test_filters_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread -k "median or sap" > gpurun_out/mta/pt_$t.log 2>&1 || { tail -20 gpurun_out/mta/pt_$t.log; exit 1; }
  echo "tile=$t tests: $(tail -1 gpurun_out/mta/pt_$t.log)"
done
for op in median3 median5 cfg3; do
  for t in 1 0 1 0; do
    IDN_MEDIAN_TILE=$t timeout -k 10 120 python bench.py --op $op --no-cpu --no-copy --steps 30 --warmup 3 > gpurun_out/mta/b_${op}_$t.json || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'tile', sys.argv[3], d['ms_per_step'])" gpurun_out/mta/b_${op}_$t.json $op $t
  done
done
