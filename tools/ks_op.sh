#!/bin/bash
# kernel-trace stats of one bench op: bash tools/ks_op.sh <out_dir> <op> [steps]
set -u
OUT=gpurun_out/$1; OP=$2; STEPS=${3:-20}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/ks" -o k --output-format csv \
  -- python3 bench.py --op "$OP" --no-cpu --no-copy --steps "$STEPS" --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
python3 - "$OUT" <<'PY'
import csv, json, sys
out = sys.argv[1]
rows = list(csv.DictReader(open(out + "/ks/k_kernel_stats.csv")))
for r in rows[:25]:
    print(f"{r['Name'][:70]:70s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1e3:9.1f} us total {float(r['TotalDurationNs'])/1e3:10.1f} us")
d = json.loads(open(out + "/bench.json").read().strip().splitlines()[-1])
print("ms_per_step", d["ms_per_step"])
PY
