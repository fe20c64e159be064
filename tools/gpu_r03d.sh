#!/bin/bash
# Round-3 A/B batch: bior1.5 synthesis forms, Gaussian NT stores (tuning build), bilateral staging.
#   bash tools/gpu_r03d.sh <out_dir>
set -u
OUT=gpurun_out/${1:-r03d}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_filters_gpu.py tests/test_configs_gpu.py -k "bilateral or cfg4 or config4" -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_bl.txt" 2>&1 || { tail -30 "$OUT/pytest_bl.txt"; exit 1; }
tail -1 "$OUT/pytest_bl.txt"
for rep in 1 2; do
  timeout -k 10 120 python bench.py --op bilateral --no-cpu --no-copy >> "$OUT/bl.jsonl" 2>> "$OUT/ab.err" || exit 1
done
for rep in 1 2 3; do
  timeout -k 10 120 python bench.py --op gauss5 --no-cpu --no-copy >> "$OUT/g5.jsonl" 2>> "$OUT/ab.err" || exit 1
  IDN_STENCIL_NTS=1 timeout -k 10 120 python bench.py --op gauss5 --lib tuning --no-cpu --no-copy >> "$OUT/g5nts.jsonl" 2>> "$OUT/ab.err" || exit 1
done
python3 - "$OUT" <<'PY'
import json, sys
for f in ("bl", "g5", "g5nts"):
    v = [json.loads(l)["roofline"] for l in open(f"{sys.argv[1]}/{f}.jsonl")]
    print(f, [("%.4f ms" % r["kernel_ms_avg"], r["frac"]) for r in v])
PY
bash tools/wl_synth_ab.sh "${1:-r03d}/wl"
