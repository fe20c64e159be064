#!/bin/bash
# bior1.5 synthesis-form A/B (IDN_WAVELET_SSTREAM through the tuning build): the form test, then
# interleaved bench lines per form and rocprofv3 kernel stats of the tiled level-1 form.
#   bash tools/wl_synth_ab.sh <out_dir>
set -u
OUT=gpurun_out/${1:-wl_synth_ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_wavelet_gpu.py -k "synthesis_forms or fp32_synthesis" -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest.txt" 2>&1 || { tail -30 "$OUT/pytest.txt"; exit 1; }
tail -2 "$OUT/pytest.txt"
for rep in 1 2; do
  for f in 3 2 1 0 3f 2f 1f; do
    IDN_WAVELET_S32=$([ "${f: -1}" = f ] && echo 1 || echo 0) IDN_WAVELET_SSTREAM=${f%f} timeout -k 10 120 python bench.py --op wavelet_bior15 --lib tuning --no-cpu --no-copy \
        >> "$OUT/ab_$f.jsonl" 2>> "$OUT/ab.err" || { tail "$OUT/ab.err"; exit 1; }
  done
done
python3 - "$OUT" <<'PY'
import json, sys
for f in "3 2 1 0 3f 2f 1f".split():
    v = [json.loads(l)["roofline"]["kernel_ms_avg"] for l in open(f"{sys.argv[1]}/ab_{f}.jsonl")]
    print("SSTREAM", f, ["%.3f" % x for x in v])
PY
IDN_WAVELET_S32=1 IDN_WAVELET_SSTREAM=3 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/ks" -o k --output-format csv \
  -- python3 bench.py --op wavelet_bior15 --lib tuning --no-cpu --no-copy --steps 20 --warmup 3 > "$OUT/ks.log" 2>&1 || { tail "$OUT/ks.log"; exit 1; }
python3 - "$OUT/ks/k_kernel_stats.csv" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:9]:
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us {float(r['Percentage']):5.1f}%")
PY
