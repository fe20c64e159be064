#!/bin/bash
# Round-2 measurement on the GPU box, steady state (bench.py's 0.5 s settle before every timed
# region): GPU parity tests, the headline bench line, one bench line per op / config, the
# rocprofv3 kernel-trace summary of the headline command, and the PMC traffic passes.
#   bash tools/profile_round2.sh <name> [ops...]
# Each GPU step runs under its own time limit; the script stops at the first failure.
set -u
R=${1:-r02f}
shift || true
OPS=${*:-"gauss3 box3 median3 median5 bilateral noise_gaussian noise_sap noise_poisson wavelet_haar3 wavelet_bior15 quant7 gauss5_blob jpeg_decode cfg2 cfg3 cfg4 cfg5"}
OUT=gpurun_out/$R
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
step() {  # step <secs> <name> <cmd...>
  local secs=$1 name=$2; shift 2
  echo "=== [$name] $*"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== [$name] rc=$rc"; tail -n 3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
step 600 pytest_gpu python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step 300 bench_default python bench.py
for op in $OPS; do
  timeout -k 10 200 python bench.py --op "$op" --no-cpu --no-copy --steps 50 --warmup 5 \
    >> "$OUT/bench_ops.jsonl" 2> "$OUT/bench_$op.err" || { echo "bench $op failed"; tail -20 "$OUT/bench_$op.err"; exit 1; }
  echo "bench $op ok"
done
step 300 prof_headline rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof_headline" -o k --output-format csv -- python3 bench.py --no-cpu
step 120 pmc_fetch rocprofv3 --pmc FETCH_SIZE -d "$ROOT/$OUT/pmc_fetch" -o pmc --output-format csv -- python3 bench.py --no-cpu --no-copy --steps 5 --warmup 2 --settle-s 0
step 120 pmc_write rocprofv3 --pmc WRITE_SIZE -d "$ROOT/$OUT/pmc_write" -o pmc --output-format csv -- python3 bench.py --no-cpu --no-copy --steps 5 --warmup 2 --settle-s 0
echo done
