#!/bin/bash
# bilateral rows-per-thread A/B (round 2; the IDN_BILATERAL_RPT knob it sets was removed after
# this measurement: RPT 5 / 6 were slower, profiles/r02/bilateral_rpt/): parity tests, bench lines
set -u
mkdir -p gpurun_out/blr
for r in 5 6; do
  IDN_BILATERAL_RPT=$r timeout -k 10 200 python -u -m pytest tests/test_filters_gpu.py -x -q --timeout 120 --timeout-method thread -k bilateral > gpurun_out/blr/pt_$r.log 2>&1 || { tail -20 gpurun_out/blr/pt_$r.log; exit 1; }
  echo "rpt=$r tests: $(tail -1 gpurun_out/blr/pt_$r.log)"
done
for r in 4 5 6 4 5 6; do
  IDN_BILATERAL_RPT=$r timeout -k 10 120 python bench.py --op bilateral --no-cpu --no-copy --steps 30 --warmup 3 > gpurun_out/blr/b_$r.json || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('rpt', sys.argv[2], d['ms_per_step'])" gpurun_out/blr/b_$r.json $r
done
