#!/bin/bash
# round 4 record: every bench op on the current code (no CPU leg), then the default headline line
# (CPU baseline + copy ceilings) and its rocprofv3 kernel stats.   bash tools/gpu/gpu_r04o.sh
set -u
OUT=gpurun_out/r04o
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/bench_ops.sh r04o ${OPS:-gauss5 gauss3 box3 median5 median3 bilateral noise_gaussian \
  noise_sap noise_poisson wavelet_haar3 wavelet_bior15 wavelet_bior15_f64 gauss5_blob quant7 cfg2 \
  cfg2p cfg3 cfg4 cfg5 jpeg_decode detect_e2e} || exit 1
timeout -k 10 300 python bench.py > "$OUT/default.json" 2> "$OUT/default.err" || exit 1
cat "$OUT/default.json"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/ks_default" -o k --output-format csv \
    -- python3 bench.py --no-cpu > "$OUT/ks_default.json" 2>&1 || exit 1
python3 -c "
import csv
for r in list(csv.DictReader(open('$OUT/ks_default/k_kernel_stats.csv')))[:3]: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,2))"
echo ok
