#!/bin/bash
# one jpeg_decode step's timeline: kernel + HIP API + memory-copy traces (no counters)
set -u
OUT=gpurun_out/r04jt
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace -d "$OUT/tr" -o t \
    --output-format csv -- python3 bench.py --op jpeg_decode --no-cpu --no-copy --steps 4 --warmup 2 \
    > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
ls -R "$OUT/tr" | head -20
