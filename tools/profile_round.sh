#!/bin/bash
# Round measurement on the GPU box: GPU parity tests, bench lines, rocprofv3 kernel stats, PMC
# traffic passes.
#   bash tools/profile_round.sh r01b [quick]
# Each GPU step runs under its own time limit; the script stops at the first failure.
# 'quick' skips the per-op stats passes.
set -u
R=${1:-r01}
MODE=${2:-full}
OUT=gpurun_out/$R
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
step() {  # step <secs> <name> <cmd...>
  local secs=$1 name=$2; shift 2
  echo "=== [$name] $*"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== [$name] rc=$rc"; tail -n 5 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
step 600 pytest_gpu python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step 400 bench_gauss5 python bench.py
OPS="box3 gauss3 median3 median5 bilateral noise_gaussian wavelet_haar3 cfg2 cfg3 cfg4 cfg5"
for op in $OPS; do
  step 300 bench_$op python bench.py --op $op --no-cpu --steps 20 --warmup 5
done
step 400 prof_stats rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o stats --output-format csv -- python3 bench.py --no-cpu --steps 20 --warmup 5
if [ "$MODE" = full ]; then
  for op in median3 median5 bilateral box3 noise_gaussian wavelet_haar3 cfg3 cfg4 cfg5; do
    step 300 prof_stats_$op rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof_$op" -o stats --output-format csv -- python3 bench.py --op $op --no-cpu --steps 10 --warmup 3
  done
fi
step 120 pmc_fetch rocprofv3 --pmc FETCH_SIZE -d "$ROOT/$OUT/pmc_fetch" -o pmc --output-format csv -- python3 bench.py --no-cpu --steps 5 --warmup 2
step 120 pmc_write rocprofv3 --pmc WRITE_SIZE -d "$ROOT/$OUT/pmc_write" -o pmc --output-format csv -- python3 bench.py --no-cpu --steps 5 --warmup 2
echo done
