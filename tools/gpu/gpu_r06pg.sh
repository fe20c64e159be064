#!/bin/bash
# round 6: Haar L3 synthesis in XCD-contiguous order (IDN_H3S_XCD=1): kernel time and FETCH_SIZE
set -u
OUT=gpurun_out/r06pg
mkdir -p $OUT
export TMPDIR=/tmp
L=image-denoising_amd/idn/libidn_hip.so
bash tools/ab_kern.sh wavelet_haar3 $OUT/k wl_h3_synth h3prod h3x1 h3prod h3x1 || exit 1
for v in h3prod h3x1; do
  cp ab/$v.so $L || exit 1
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d "$(pwd)/$OUT/f_$v" -o pmc --output-format csv \
    -- python3 bench.py --op wavelet_haar3 --no-cpu --no-copy --steps 3 --warmup 1 --settle-s 0 > $OUT/f_$v.log 2>&1 || exit 1
  python3 - $OUT/f_$v $v <<'PY'
import csv, glob, sys
v = []
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'wl_h3_synth' in r['Kernel_Name']: v.append(float(r['Counter_Value']))
print(sys.argv[2], 'synth FETCH_SIZE x2 MB', round(2 * 1024 * sum(v) / len(v) / 1e6, 1))
PY
done
cp ab/new.so $L
