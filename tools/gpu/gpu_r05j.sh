#!/bin/bash
# round 5: checkpointed JPEG entropy passes -- parity, then decode / e2e timing and timeline
set -u
OUT=gpurun_out/${1:-r05j}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_jpeg_gpu.py tests/test_minibatch_gpu.py -x -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.txt" 2>&1 \
    || { tail -40 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
for op in jpeg_decode detect_e2e; do
  timeout -k 10 300 python bench.py --op $op --no-cpu --no-copy --steps 30 --warmup 5 \
    > "$OUT/$op.json" 2>> "$OUT/bench.err" || exit 1
  echo "$op $(grep -ho '"ms_per_step": [0-9.]*' $OUT/$op.json)"
done
timeout -k 10 300 python tools/e2e_stages.py --iters 200 --out "$OUT/e2e_stages.json" \
  > "$OUT/e2e.log" 2>&1 || { tail -20 "$OUT/e2e.log"; exit 1; }
cat "$OUT/e2e_stages.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$(pwd)/$OUT/e2e_prof" \
  -o k --output-format csv -- python3 bench.py --op detect_e2e --no-cpu --no-copy --steps 30 \
  --warmup 5 > "$OUT/e2e_prof.log" 2>&1 || { tail -20 "$OUT/e2e_prof.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$(pwd)/$OUT/jpeg_prof" \
  -o k --output-format csv -- python3 bench.py --op jpeg_decode --no-cpu --no-copy --steps 10 \
  --warmup 3 > "$OUT/jpeg_prof.log" 2>&1 || { tail -20 "$OUT/jpeg_prof.log"; exit 1; }
echo ok
