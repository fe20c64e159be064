#!/bin/bash
# rocprofv3 PMC passes over `bench.py --op <op>`, one run per counter group (groups separated by
# ';'), each under its own limit; stops at the first failure.  Summaries: tools/pmc_summary.py.
#   bash tools/pmc_pass.sh <out_dir> <op> "<counters>;<counters>;..."
set -u
OUT=gpurun_out/$1; OP=$2; GROUPS_=$3
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
i=0
IFS=';' read -ra G <<< "$GROUPS_"
for g in "${G[@]}"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $g -d "$ROOT/$OUT/pmc_${OP}_$i" -o pmc --output-format csv \
    -- python3 bench.py --op "$OP" --no-cpu --no-copy --steps 3 --warmup 1 --settle-s 0 > "$OUT/pmc_${OP}_$i.log" 2>&1 || { tail "$OUT/pmc_${OP}_$i.log"; exit 1; }
done
python3 tools/pmc_summary.py "$OUT"/pmc_${OP}_* > "$OUT/pmc_${OP}.txt" && cat "$OUT/pmc_${OP}.txt"
