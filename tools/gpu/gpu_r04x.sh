#!/bin/bash
# round 4: adaptive default JPEG chunk size -- JPEG / drop-in tests, then the per-image end-to-end
# op and the batch decode op with kernel stats.   bash tools/gpu/gpu_r04x.sh
set -u
OUT=gpurun_out/r04x
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_jpeg_gpu.py tests/test_minibatch_gpu.py -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.txt" 2>&1
rc=$?
tail -2 "$OUT/pytest.txt"
[ $rc = 0 ] || exit $rc
bash tools/ks_op.sh r04x/e2e detect_e2e 20 || exit 1
bash tools/ks_op.sh r04x/jpeg jpeg_decode 10 || exit 1
echo ok
