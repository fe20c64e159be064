#!/bin/bash
# Closing measurement of the round: whole GPU suite, smoke(), the default bench line, every op's
# bench line (no CPU leg), and rocprofv3 kernel stats of the headline and the pipelines.
#   bash tools/final_r03.sh <out_dir>
set -u
OUT=gpurun_out/${1:-final_r03}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest_gpu.txt" 2>&1
rc=$?
tail -2 "$OUT/pytest_gpu.txt"; grep -E "^FAILED" "$OUT/pytest_gpu.txt" | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1 || { tail "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
timeout -k 10 300 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { tail "$OUT/bench_default.err"; exit 1; }
for op in gauss5 gauss3 box3 median3 median5 bilateral noise_gaussian noise_sap noise_poisson wavelet_haar3 wavelet_bior15 gauss5_blob quant7 cfg2 cfg3 cfg4 cfg5 jpeg_decode detect_e2e; do
  timeout -k 10 200 python bench.py --op $op --no-cpu --no-copy >> "$OUT/bench_ops.jsonl" 2> "$OUT/bench_$op.err" || { echo "bench $op failed"; tail -5 "$OUT/bench_$op.err"; exit 1; }
done
python3 - "$OUT/bench_ops.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]
    print(f"{d['config']['op']:16s} ms/step {d['ms_per_step']:.4f} kern {r['kernel_ms_avg']:.4f} frac {r['frac']}")
PY
for op in gauss5 cfg4 cfg5 wavelet_bior15; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/ks_$op" -o k --output-format csv \
    -- python3 bench.py --op $op --no-cpu --no-copy > "$OUT/ks_$op.log" 2>&1 || { tail "$OUT/ks_$op.log"; exit 1; }
done
echo done
