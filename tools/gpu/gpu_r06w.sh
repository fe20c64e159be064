#!/bin/bash
# round 6: ImageReader windows -- reader test, detect_e2e vs detect_e2e_pipelined at read windows
# 1/2/4/8/16, a merged timeline of a pipelined step
set -u
OUT=gpurun_out/r06w
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_jpeg_gpu.py -x -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider -k "image_reader or imread_gpu" > $OUT/pytest.txt 2>&1
rc=$?; tail -3 $OUT/pytest.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python bench.py --op detect_e2e --no-cpu --no-copy --steps 200 --warmup 20 >> $OUT/bench.jsonl 2> $OUT/bench.err || exit 1
for b in 1 2 4 8 16; do
  IDN_BENCH_READ_BATCH=$b timeout -k 10 200 python bench.py --op detect_e2e_pipelined --no-cpu --no-copy --steps 400 --warmup 40 >> $OUT/bench.jsonl 2> $OUT/bench.err || exit 1
  python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1])][-1]; print(sys.argv[2], d['config']['op'], d['ms_per_step'])" $OUT/bench.jsonl $b | tee -a $OUT/sweep.txt
done
timeout -k 10 240 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace -d "$(pwd)/$OUT/tr" -o t \
    --output-format csv -- python3 bench.py --op detect_e2e_pipelined --no-cpu --no-copy --steps 24 --warmup 16 --settle-s 0 \
    > $OUT/tr_bench.json 2> $OUT/tr_bench.err || exit 1
python3 tools/e2e_timeline.py $OUT/tr ycc_keys_init 3 > $OUT/timeline.txt || exit 1
tail -1 $OUT/timeline.txt
