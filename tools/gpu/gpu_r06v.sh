#!/bin/bash
# round 6: ImageReader (next image decoded ahead) -- JPEG tests, detect_e2e and detect_e2e_pipelined
# bench lines, stage breakdown, a merged timeline of a pipelined step
set -u
OUT=gpurun_out/r06v
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_jpeg_gpu.py -x -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest.txt 2>&1
rc=$?; tail -3 $OUT/pytest.txt; [ $rc = 0 ] || exit $rc
for op in detect_e2e detect_e2e_pipelined detect_e2e detect_e2e_pipelined; do
  timeout -k 10 200 python bench.py --op $op --no-cpu --no-copy --steps 200 --warmup 20 >> $OUT/bench.jsonl 2> $OUT/bench.err || exit 1
  python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1])][-1]; print(d['config']['op'], d['ms_per_step'], d.get('ms_per_image'))" $OUT/bench.jsonl
done
timeout -k 10 240 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace -d "$(pwd)/$OUT/tr" -o t \
    --output-format csv -- python3 bench.py --op detect_e2e_pipelined --no-cpu --no-copy --steps 8 --warmup 4 --settle-s 0 \
    > $OUT/tr_bench.json 2> $OUT/tr_bench.err || exit 1
python3 tools/e2e_timeline.py $OUT/tr jpeg_unstuff_count 3 > $OUT/timeline.txt || exit 1
tail -1 $OUT/timeline.txt
