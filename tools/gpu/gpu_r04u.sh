#!/bin/bash
# round 4: bior1.5 analysis with 256-thread strips whose LDS is sized for them (4 workgroups per
# CU) against the 512-thread product, tuning build, kernel stats per config.  bash tools/gpu/gpu_r04u.sh
set -u
OUT=gpurun_out/r04u
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
print(f"{sys.argv[2]:24s} level1 {l1:8.1f} deeper {deep:7.1f}")
PY
}
run default IDN_X=0 || exit 1
run wst256 IDN_WAVELET_WST=256 || exit 1
for b in 1 2 3 4; do run wst256_b$b IDN_WAVELET_WST=256 IDN_WAVELET_BANDS=$((b + 256 * b + 65536 * b)) || exit 1; done
run default2 IDN_X=0 || exit 1
echo ok
