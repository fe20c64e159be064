#!/bin/bash
set -u
OUT=gpurun_out/r03j
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_filters_gpu.py -k "tile_fetch or gaussian or box or blob" -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest.txt" 2>&1 || { tail -30 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
for rep in 1 2 3; do
  timeout -k 10 120 python bench.py --op gauss5 --no-cpu --no-copy >> "$OUT/g1.jsonl" 2>> "$OUT/ab.err" || exit 1
  IDN_STENCIL_GLDS=2 timeout -k 10 120 python bench.py --op gauss5 --lib tuning --no-cpu --no-copy >> "$OUT/g2.jsonl" 2>> "$OUT/ab.err" || exit 1
  IDN_STENCIL_GLDS=0 timeout -k 10 120 python bench.py --op gauss5 --lib tuning --no-cpu --no-copy >> "$OUT/g0.jsonl" 2>> "$OUT/ab.err" || exit 1
done
for f in g1 g2 g0; do echo "$f $(grep -ho '"frac": [0-9.]*' "$OUT/$f.jsonl" | tr '\n' ' ')"; done
for v in 0 2; do
  IDN_STENCIL_GLDS=$v timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
    -d "$ROOT/$OUT/pmc_glds$v" -o pmc --output-format csv -- python3 bench.py --op gauss5 --lib tuning --no-cpu --no-copy --steps 3 --warmup 1 --settle-s 0 > "$OUT/pmc_glds$v.log" 2>&1 || { tail "$OUT/pmc_glds$v.log"; exit 1; }
done
IDN_STENCIL_GLDS=2 timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d "$ROOT/$OUT/pmc_fetch2" -o pmc --output-format csv -- python3 bench.py --op gauss5 --lib tuning --no-cpu --no-copy --steps 3 --warmup 1 --settle-s 0 > "$OUT/pmc_fetch2.log" 2>&1 || { tail "$OUT/pmc_fetch2.log"; exit 1; }
python3 tools/pmc_summary.py --match stencil_u8 "$OUT"/pmc_glds0 > "$OUT/pmc_glds0.txt"; python3 tools/pmc_summary.py --match stencil_u8 "$OUT"/pmc_glds2 "$OUT"/pmc_fetch2 > "$OUT/pmc_glds2.txt"; cat "$OUT"/pmc_glds*.txt
