#!/bin/bash
# round 5: the live path's fused colour range -- parity, the live-path A/B, the e2e breakdown
set -u
OUT=${1:-r05h}
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python -u -m pytest tests/test_live_path_gpu.py tests/test_pipeline_gpu.py \
    tests/test_wavelet_gpu.py tests/test_noise_gpu.py -x -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/$OUT/pytest.txt 2>&1 \
    || { tail -40 gpurun_out/$OUT/pytest.txt; exit 1; }
tail -1 gpurun_out/$OUT/pytest.txt
for rep in 1 2; do
  for op in live_f64 live_f64_unfused wavelet_bior15_f64; do
    timeout -k 10 200 python bench.py --op $op --no-cpu --no-copy --steps 20 --warmup 3 \
      >> gpurun_out/$OUT/$op.jsonl 2>> gpurun_out/$OUT/bench.err || exit 1
  done
done
for op in live_f64 live_f64_unfused wavelet_bior15_f64; do
  echo "$op $(grep -ho '"ms_per_step": [0-9.]*' gpurun_out/$OUT/$op.jsonl | tr '\n' ' ')"
done
timeout -k 10 300 python tools/e2e_stages.py --iters 200 --out gpurun_out/$OUT/e2e_stages.json \
  > gpurun_out/$OUT/e2e.log 2>&1 || { tail -20 gpurun_out/$OUT/e2e.log; exit 1; }
cat gpurun_out/$OUT/e2e_stages.json
