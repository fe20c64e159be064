#!/bin/bash
# whole GPU suite, then bench lines of the round-3 kernels
set -u
OUT=gpurun_out/${1:-r03h}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest.txt" 2>&1
rc=$?
tail -3 "$OUT/pytest.txt"
grep -E "^FAILED" "$OUT/pytest.txt" | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
for op in gauss5 gauss5_blob gauss5 wavelet_bior15 bilateral gauss5; do
  timeout -k 10 200 python bench.py --op $op --no-cpu --steps 20 --warmup 5 >> "$OUT/bench.jsonl" 2> "$OUT/bench_$op.err" || { tail -5 "$OUT/bench_$op.err"; exit 1; }
done
python3 - "$OUT/bench.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]
    print(f"{d['config']['op']:16s} ms/step {d['ms_per_step']:.4f} kern {r['kernel_ms_avg']:.4f} frac {r['frac']} copy-frac {r.get('frac_of_default_policy_copy')}")
PY
cp image-denoising_amd/idn/libidn_hip.so ab/prod.so
bash tools/ab_lib.sh wavelet_bior15 "$OUT/pf" new pf1 chist new pf1 chist
cp ab/prod.so image-denoising_amd/idn/libidn_hip.so
