#!/bin/bash
# Round-3 measurements: Gaussian store-policy A/B, per-kernel stats + SQ PMC of bior1.5 and
# bilateral (the "before" of their rework).  Every GPU step under its own limit; stops on failure.
set -u
OUT=gpurun_out/${1:-r03b}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
for rep in 1 2 3; do
  timeout -k 10 120 python bench.py --op gauss5 --no-cpu --no-copy >> "$OUT/ab_gauss5.jsonl" 2>> "$OUT/ab.err" || exit 1
  IDN_STENCIL_NTS=1 timeout -k 10 120 python bench.py --op gauss5 --lib tuning --no-cpu --no-copy >> "$OUT/ab_gauss5_nts.jsonl" 2>> "$OUT/ab.err" || exit 1
done
python - "$OUT" <<'PY'
import json, sys
for f in ("ab_gauss5", "ab_gauss5_nts"):
    v = [json.loads(l)["roofline"]["frac"] for l in open(f"{sys.argv[1]}/{f}.jsonl")]
    print(f, v)
PY
for op in wavelet_bior15 bilateral; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/ks_$op" -o k --output-format csv \
    -- python3 bench.py --op $op --no-cpu --no-copy --steps 20 --warmup 3 > "$OUT/ks_$op.log" 2>&1 || { tail "$OUT/ks_$op.log"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
    -d "$ROOT/$OUT/pmc_$op" -o pmc --output-format csv -- python3 bench.py --op $op --no-cpu --no-copy --steps 3 --warmup 1 --settle-s 0 > "$OUT/pmc_$op.log" 2>&1 || { tail "$OUT/pmc_$op.log"; exit 1; }
done
echo done
