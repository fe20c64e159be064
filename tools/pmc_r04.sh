#!/bin/bash
# Round-4 counter evidence: per op a kernel-trace stats run and four rocprofv3 --pmc passes
# (FETCH_SIZE; WRITE_SIZE; two groups of 8 SQ counters), each under its own time limit; stops at
# the first failure.  Fold with tools/pmc_r04.py.   bash tools/pmc_r04.sh <out_dir> <op> ...
set -u
OUT=gpurun_out/$1
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
S1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
S2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for op in "$@"; do
  mkdir -p "$OUT/$op"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/$op/ks" -o k --output-format csv \
    -- python3 bench.py --op "$op" --no-cpu --no-copy --steps 10 --warmup 2 > "$OUT/$op/ks.log" 2>&1 \
    || { tail -5 "$OUT/$op/ks.log"; exit 1; }
  for pass in fetch write sq1 sq2; do
    case $pass in
      fetch) C="FETCH_SIZE" ;;
      write) C="WRITE_SIZE" ;;
      sq1) C="$S1" ;;
      sq2) C="$S2" ;;
    esac
    timeout -s KILL 90 rocprofv3 --pmc $C -d "$ROOT/$OUT/$op/$pass" -o pmc --output-format csv \
      -- python3 bench.py --op "$op" --no-cpu --no-copy --steps 3 --warmup 1 --settle-s 0 \
      > "$OUT/$op/$pass.log" 2>&1 || { tail -5 "$OUT/$op/$pass.log"; exit 1; }
  done
  echo "$op done"
done
echo ok
