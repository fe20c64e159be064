#!/bin/bash
# round 4: bior1.5 analysis strip width x band count sweep (tuning build: IDN_WAVELET_WST threads
# per strip, IDN_WAVELET_BANDS level-1 bands) -- kernel stats per config; and the product with
# the reverted band query.  bash tools/gpu/gpu_r04f.sh
set -u
OUT=gpurun_out/r04f
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/ks_$name" -o k --output-format csv \
    -- python3 bench.py --op wavelet_bior15 --lib tuning --no-cpu --no-copy --steps 10 --warmup 2 > /dev/null 2>&1 || return 1
  python3 - "$OUT/ks_$name/k_kernel_stats.csv" "$name" <<'PY'
import csv, sys
rows = {r['Name'].split('(')[0]: float(r['AverageNs']) / 1e3 for r in csv.DictReader(open(sys.argv[1]))}
l1 = sum(v for k, v in rows.items() if 'wl_dwt_stream<0' in k)
deep = sum(v for k, v in rows.items() if 'wl_dwt_stream<3' in k)
tot = sum(v for k, v in rows.items() if 'idn::' in k)
print(f"{sys.argv[2]:24s} level1 {l1:8.1f} deeper {deep:7.1f} total {tot:8.1f}")
PY
}
run default IDN_X=0 || exit 1
for b in 1 2 4 8; do run wst64_b$b IDN_WAVELET_WST=64 IDN_WAVELET_BANDS=$b || exit 1; done
for b in 1 2 4; do run wst128_b$b IDN_WAVELET_WST=128 IDN_WAVELET_BANDS=$b || exit 1; done
for b in 1 2; do run wst256_b$b IDN_WAVELET_WST=256 IDN_WAVELET_BANDS=$b || exit 1; done
for b in 2 4; do run wst512_b$b IDN_WAVELET_BANDS=$b || exit 1; done
echo ok
