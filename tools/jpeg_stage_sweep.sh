#!/bin/bash
# JPEG staging sweep: host gather threads x H2D parts (bench op jpeg_decode, steady state)
#   bash tools/jpeg_stage_sweep.sh <out_dir> "t1,p1 t2,p2 ..."
set -u
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for tp in $1; do
  t=${tp%,*}; p=${tp#*,}
  IDN_JPEG_THREADS=$t IDN_JPEG_PARTS=$p timeout -k 10 200 python bench.py --op jpeg_decode --no-cpu --no-copy --steps 30 --warmup 3 > "$OUT/t${t}_p${p}.json" 2> "$OUT/t${t}_p${p}.err" || { tail -5 "$OUT/t${t}_p${p}.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'])" "$OUT/t${t}_p${p}.json" "threads=$t parts=$p"
done
