#!/bin/bash
# rocprofv3 kernel-trace summaries of bench ops, one profiler run per op (run on the GPU box):
#   bash tools/profile_ops.sh <out_dir> op1 op2 ...
# writes <out_dir>/<op>/k_kernel_stats.csv and <out_dir>/<op>.jsonl (the bench line of that run)
set -o pipefail
OUT=$1
shift
export TMPDIR=/tmp
mkdir -p "$OUT"
for op in "$@"; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/$op" -o k --output-format csv \
    -- python bench.py --op "$op" --no-cpu --no-copy --steps 20 --warmup 5 \
    > "$OUT/$op.jsonl" 2> "$OUT/$op.err" || { tail -20 "$OUT/$op.err"; exit 1; }
  echo "$op done"
done
