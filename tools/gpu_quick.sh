#!/bin/bash
# Quick GPU check: selected pytest files then bench lines for the given ops.
#   bash tools/gpu_quick.sh <out_dir> "<pytest files>" "<ops>"
set -u
OUT=gpurun_out/$1; TESTS=$2; OPS=$3
mkdir -p "$OUT"
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { tail -30 "$OUT/pytest.txt"; exit 1; }
  tail -2 "$OUT/pytest.txt"
fi
for op in $OPS; do
  timeout -k 10 200 python bench.py --op $op --no-cpu --steps 20 --warmup 5 >> "$OUT/bench.jsonl" 2> "$OUT/bench_$op.err" || { tail -20 "$OUT/bench_$op.err"; exit 1; }
done
python - "$OUT/bench.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]
    print(f"{d['config']['op']:16s} ms/step {d['ms_per_step']:.4f} kern {r['kernel_ms_avg']:.4f} frac {r['frac']:.3f}")
PY
