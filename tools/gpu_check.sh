#!/bin/bash
# GPU check: the -m gpu suite (or a subset), then bench lines for the given ops.
#   bash tools/gpu_check.sh <out_dir> "<pytest args or ->" "<ops>" [steps]
set -u
OUT=gpurun_out/$1; TESTS=$2; OPS=$3; STEPS=${4:-20}
mkdir -p "$OUT"
if [ "$TESTS" != "-" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -q --timeout 120 --timeout-method thread \
      -p no:cacheprovider > "$OUT/pytest.txt" 2>&1
  rc=$?
  tail -25 "$OUT/pytest.txt"
  # a crash / abort / timeout of the test process ends the GPU work of this call
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
for op in $OPS; do
  timeout -k 10 300 python bench.py --op $op --no-cpu --steps $STEPS --warmup 5 >> "$OUT/bench.jsonl" \
      2> "$OUT/bench_$op.err" || { echo "bench $op failed"; tail -20 "$OUT/bench_$op.err"; exit 1; }
done
if [ -n "$OPS" ]; then
python - "$OUT/bench.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]
    fr = r["frac"]
    print(f"{d['config']['op']:16s} ms/step {d['ms_per_step']:.4f} kern {r['kernel_ms_avg']:.4f} "
          f"frac {fr if fr is None else round(fr, 3)} " + (f"ms/img {d['ms_per_image']}" if 'ms_per_image' in d else ""))
PY
fi
