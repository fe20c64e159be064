#!/bin/bash
# round 6: wl_h3_stats timing probes (parts removed; wrong results) -- which part costs what
set -u
OUT=gpurun_out/r06g
mkdir -p $OUT
for rep in 1 2; do bash tools/ab_lib.sh wavelet_haar3 $OUT/ab$rep p1 p2 p4 p8 p15 new | grep -v "^ok" || exit 1; done
python3 - <<'PY'
import csv,glob
for f in glob.glob('gpurun_out/r06g/ab2/prof_new/*kernel_stats.csv'):
    for r in csv.DictReader(open(f)):
        if 'idn' in r['Name']: print(r['Name'][:40], round(float(r['AverageNs'])/1e3,1))
PY
