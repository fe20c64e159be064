#!/bin/bash
# round 6: pinned host copies for the blobs -- blob/detect GPU tests, detect_e2e and the read-ahead loop
set -u
OUT=gpurun_out/r06x
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider -k "blob or detect or image_reader" > $OUT/pytest.txt 2>&1
rc=$?; tail -3 $OUT/pytest.txt; [ $rc = 0 ] || exit $rc
for op in detect_e2e detect_e2e_pipelined detect_e2e detect_e2e_pipelined; do
  timeout -k 10 200 python bench.py --op $op --no-cpu --no-copy --steps 400 --warmup 40 >> $OUT/bench.jsonl 2> $OUT/bench.err || exit 1
  python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1])][-1]; print(d['config']['op'], d['ms_per_step'])" $OUT/bench.jsonl
done
timeout -k 10 200 python tools/e2e_stages.py --out $OUT/e2e_stages.json > $OUT/e2e_stages.txt 2>&1 || exit 1
tail -4 $OUT/e2e_stages.txt
