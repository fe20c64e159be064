#!/bin/bash
# bilateral A/B: shared own-output weights (IDN_BL2_SYM=1) vs every tap looked up (0), both in
# the tuning build, after the bilateral GPU tests.  bash tools/bl_sym_ab.sh <out_dir>
set -u
OUT=gpurun_out/${1:-bl_sym_ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_filters_gpu.py -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider -k bilateral > "$OUT/pytest.txt" 2>&1 || { tail -30 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
for rep in 1 2; do
  timeout -k 10 120 python bench.py --op bilateral --no-cpu --no-copy >> "$OUT/ab_prod.jsonl" 2>> "$OUT/ab.err" || exit 1
  for s in 1 0; do
    IDN_BL2_SYM=$s timeout -k 10 120 python bench.py --op bilateral --lib tuning --no-cpu --no-copy >> "$OUT/ab_sym$s.jsonl" 2>> "$OUT/ab.err" || exit 1
  done
done
for f in prod sym1 sym0; do echo "$f $(grep -ho '"kernel_ms_avg": [0-9.]*' "$OUT/ab_$f.jsonl" | tr '\n' ' ')"; done
