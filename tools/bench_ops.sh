#!/bin/bash
# bench lines (no CPU leg) for the given ops into gpurun_out/<dir>/bench.jsonl, one summary line each
#   bash tools/bench_ops.sh <dir> op1 op2 ...
set -u
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for op in "$@"; do
  timeout -k 10 200 python bench.py --op $op --no-cpu --no-copy --steps 20 --warmup 5 >> "$OUT/bench.jsonl" 2> "$OUT/bench_$op.err" || { tail -20 "$OUT/bench_$op.err"; exit 1; }
done
python - "$OUT/bench.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]
    frac = "-" if r["frac"] is None else f"{r['frac']:.3f}"
    print(f"{d['config']['op']:16s} ms/step {d['ms_per_step']:.4f} kern {r['kernel_ms_avg']:.4f} GB/s {r['achieved']:.0f} frac {frac}")
PY
