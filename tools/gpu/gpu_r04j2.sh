#!/bin/bash
# JPEG batch parts: GPU tests of the decoder, then same-run A/B of the part count (ab/p<N>.so)
set -u
OUT=gpurun_out/r04j3
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_jpeg_gpu.py -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest.txt" 2>&1
rc=$?
tail -2 "$OUT/pytest.txt"
[ $rc = 0 ] || exit $rc
bash tools/ab_e2e.sh r04j3/ab jpeg_decode p1 p2 q2 q3 q4
