#!/bin/bash
# round 6: detect_e2e single-image step -- stage breakdown and a merged kernel / HIP API / copy
# timeline of one step
set -u
OUT=gpurun_out/r06u
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/e2e_stages.py --iters 200 --out $OUT/e2e_stages.json > $OUT/stages.log 2>&1 || exit 1
tail -16 $OUT/stages.log
timeout -k 10 240 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace -d "$(pwd)/$OUT/tr" -o t \
    --output-format csv -- python3 bench.py --op detect_e2e --no-cpu --no-copy --steps 8 --warmup 4 --settle-s 0 \
    > $OUT/bench.json 2> $OUT/bench.err || exit 1
python3 tools/e2e_timeline.py $OUT/tr jpeg_unstuff_count 3 > $OUT/timeline.txt || exit 1
tail -3 $OUT/timeline.txt
