#!/bin/bash
# bior1.5 precision A/B through the tuning build: IDN_WAVELET_A32 (analysis) x IDN_WAVELET_S32
# (synthesis); the wavelet GPU tests first, then interleaved bench lines and kernel stats.
#   bash tools/wl_prec_ab.sh <out_dir> [modes]     (mode = <A32>s<S32>, e.g. 0s1)
set -u
OUT=gpurun_out/${1:-wl_prec_ab}
MODES=${2:-"0s1 1s1 2s1 3s1"}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 400 python -u -m pytest tests/test_wavelet_gpu.py -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest.txt" 2>&1 || { tail -30 "$OUT/pytest.txt"; exit 1; }
tail -2 "$OUT/pytest.txt"
for rep in 1 2; do
  for m in $MODES; do
    IDN_WAVELET_A32=${m%s*} IDN_WAVELET_S32=${m#*s} timeout -k 10 120 python bench.py --op wavelet_bior15 --lib tuning \
        --no-cpu --no-copy >> "$OUT/ab_$m.jsonl" 2>> "$OUT/ab.err" || { tail "$OUT/ab.err"; exit 1; }
  done
done
python3 - "$OUT" $MODES <<'PY'
import json, sys
for m in sys.argv[2:]:
    v = [json.loads(l)["roofline"]["kernel_ms_avg"] for l in open(f"{sys.argv[1]}/ab_{m}.jsonl")]
    print("mode", m, ["%.3f" % x for x in v])
PY
last=${MODES##* }
IDN_WAVELET_A32=${last%s*} IDN_WAVELET_S32=${last#*s} timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/ks" -o k \
  --output-format csv -- python3 bench.py --op wavelet_bior15 --lib tuning --no-cpu --no-copy --steps 20 --warmup 3 \
  > "$OUT/ks.log" 2>&1 || { tail "$OUT/ks.log"; exit 1; }
python3 - "$OUT/ks/k_kernel_stats.csv" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:9]:
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us {float(r['Percentage']):5.1f}%")
PY
