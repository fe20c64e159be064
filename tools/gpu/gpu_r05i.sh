#!/bin/bash
# round 5: detect_e2e stage breakdown and its kernel timeline; the live path's kernel stats
set -u
OUT=gpurun_out/${1:-r05i}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python tools/e2e_stages.py --iters 200 --out "$OUT/e2e_stages.json" \
  > "$OUT/e2e.log" 2>&1 || { tail -20 "$OUT/e2e.log"; exit 1; }
cat "$OUT/e2e_stages.json"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$(pwd)/$OUT/e2e_prof" \
  -o k --output-format csv -- python3 bench.py --op detect_e2e --no-cpu --no-copy --steps 30 \
  --warmup 5 > "$OUT/e2e_prof.log" 2>&1 || { tail -20 "$OUT/e2e_prof.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$(pwd)/$OUT/live_prof" -o k \
  --output-format csv -- python3 bench.py --op live_f64 --no-cpu --no-copy --steps 10 --warmup 2 \
  > "$OUT/live_prof.log" 2>&1 || { tail -20 "$OUT/live_prof.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$(pwd)/$OUT/live_unf_prof" -o k \
  --output-format csv -- python3 bench.py --op live_f64_unfused --no-cpu --no-copy --steps 10 \
  --warmup 2 > "$OUT/live_unf_prof.log" 2>&1 || { tail -20 "$OUT/live_unf_prof.log"; exit 1; }
echo ok
