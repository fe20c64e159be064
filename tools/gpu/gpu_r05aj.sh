#!/bin/bash
# round 5: kernel stats of a 256-file decode at 1536-bit chunks, old / new library
set -u
OUT=${1:-r05aj}
mkdir -p gpurun_out/$OUT
L=image-denoising_amd/idn/libidn_hip.so
cp $L gpurun_out/$OUT/keep.so
for v in old new2; do
  cp ab/$v.so $L || exit 1
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$(pwd)/gpurun_out/$OUT/ks_$v" -o k --output-format csv \
      -- python3 tools/jpeg_single.py --iters 20 --batch 256 --chunk 1536 > gpurun_out/$OUT/ks_$v.log 2>&1 || { cp gpurun_out/$OUT/keep.so $L; exit 1; }
done
cp gpurun_out/$OUT/keep.so $L
rm gpurun_out/$OUT/keep.so
for v in old new2; do
  echo "== $v"
  python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r['Name'][:60].ljust(60), r['Calls'].rjust(5), '%9.1f' % (float(r['AverageNs'])/1e3), '%10.1f' % (float(r['TotalDurationNs'])/1e3))
" gpurun_out/$OUT/ks_$v/k_kernel_stats.csv | head -14
done
