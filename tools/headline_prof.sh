#!/bin/bash
# Headline records: the default bench line, rocprofv3 --kernel-trace --stats of the same command,
# HBM traffic passes (FETCH_SIZE, WRITE_SIZE: separate runs) and one SQ pass, each under its own
# limit; then the band-height A/B of the LDS-DMA tile (ab/ variants).
#   bash tools/headline_prof.sh <out_dir>
set -u
OUT=gpurun_out/${1:-headline}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 300 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { tail "$OUT/bench_default.err"; exit 1; }
cat "$OUT/bench_default.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/ks" -o k --output-format csv \
  -- python3 bench.py --no-cpu > "$OUT/ks.log" 2>&1 || { tail "$OUT/ks.log"; exit 1; }
head -3 "$OUT/ks/k_kernel_stats.csv" | cut -c1-200
for c in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  tag=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $c -d "$ROOT/$OUT/pmc_$tag" -o pmc --output-format csv \
    -- python3 bench.py --op gauss5 --no-cpu --no-copy --steps 3 --warmup 1 --settle-s 0 > "$OUT/pmc_$tag.log" 2>&1 || { tail "$OUT/pmc_$tag.log"; exit 1; }
done
python3 tools/pmc_summary.py --match stencil_u8 "$OUT"/pmc_FETCH_SIZE "$OUT"/pmc_WRITE_SIZE "$OUT"/pmc_SQ_INSTS_VALU > "$OUT/pmc_summary.txt"
cat "$OUT/pmc_summary.txt"
bash tools/ab_lib.sh gauss5 "$OUT/nb" new nb4 nb8 nb10 new nb4 nb8 nb10
