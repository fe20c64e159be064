#!/bin/bash
# round 6: whole GPU suite on the two-read Haar-3 path, then haar3 / cfg5 bench lines + kernel trace
set -u
OUT=gpurun_out/r06j
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest.txt" 2>&1
rc=$?; tail -3 "$OUT/pytest.txt"; [ $rc = 0 ] || exit $rc
bash tools/bench_ops.sh r06j wavelet_haar3 cfg5 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$(pwd)/$OUT/ks" -o k --output-format csv \
  -- python3 bench.py --op cfg5 --no-cpu --no-copy --steps 10 --warmup 2 > "$OUT/ks.log" 2>&1 || exit 1
echo ok
