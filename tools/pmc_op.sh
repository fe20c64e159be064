#!/bin/bash
# One rocprofv3 PMC pass (8 SQ counters) over `bench.py --op <op>` per value of an environment
# knob, for instruction-mix / LDS-conflict comparisons of kernel variants.
#   bash tools/pmc_op.sh <op> <out_dir> [KNOB=v1,v2,...]
# Each pass runs under its own time limit; the script stops at the first failure.
set -u
OP=$1
OUT=$2
KNOB=${3:-}
mkdir -p "$OUT"
export TMPDIR=/tmp
COUNTERS="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
if [ -z "$KNOB" ]; then
  VALS="default"
else
  NAME=${KNOB%%=*}
  VALS=$(echo "${KNOB#*=}" | tr ',' ' ')
fi
for v in $VALS; do
  if [ "$v" != default ]; then export "$NAME=$v"; fi
  timeout -s KILL 90 rocprofv3 --pmc $COUNTERS -d "$OUT/$v" -o pmc --output-format csv \
    -- python3 bench.py --op "$OP" --no-cpu --steps 3 --warmup 1 > "$OUT/log_$v.txt" 2>&1 || exit 1
done
echo ok
