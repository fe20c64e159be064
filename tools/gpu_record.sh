#!/bin/bash
# checkpoint record (round 5 on): the whole GPU suite, smoke, every bench op (no CPU leg; detect_e2e
# with 200 steps), the default headline line and its kernel stats
set -u
OUT=gpurun_out/${1:-record}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest.txt" 2>&1
rc=$?
tail -2 "$OUT/pytest.txt"
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || exit 1
tail -1 "$OUT/smoke.txt"
bash tools/bench_ops.sh "${1:-record}" gauss5 gauss3 box3 median5 median3 bilateral noise_gaussian \
  noise_sap noise_poisson wavelet_haar3 wavelet_bior15 wavelet_bior15_f64 live_f64 live_f64_unfused \
  gauss5_blob quant7 cfg2 cfg3 cfg4 cfg5 jpeg_decode || exit 1
timeout -k 10 300 python bench.py --op detect_e2e --no-cpu --no-copy --steps 200 --warmup 20 \
  >> "$OUT/bench.jsonl" 2> "$OUT/e2e.err" || exit 1
tail -1 "$OUT/bench.jsonl"
timeout -k 10 300 python bench.py --op detect_e2e_pipelined --no-cpu --no-copy --steps 400 --warmup 40 \
  >> "$OUT/bench.jsonl" 2> "$OUT/e2e.err" || exit 1
tail -1 "$OUT/bench.jsonl"
timeout -k 10 300 python bench.py > "$OUT/default.json" 2> "$OUT/default.err" || exit 1
cat "$OUT/default.json"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$(pwd)/$OUT/ks_default" -o k \
  --output-format csv -- python3 bench.py --no-cpu > "$OUT/ks_default.log" 2>&1 || exit 1
echo ok
