#!/bin/bash
# round 4 checkpoint: the whole GPU test suite, then the bior1.5 counter passes on the product.
#   bash tools/gpu/gpu_r04m.sh
set -u
OUT=gpurun_out/r04m
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest.txt" 2>&1
rc=$?
tail -3 "$OUT/pytest.txt"
[ $rc = 0 ] || exit $rc
bash tools/pmc_r04.sh r04m/pmc wavelet_bior15 || exit 1
echo ok
