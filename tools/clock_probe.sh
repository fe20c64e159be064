#!/bin/bash
# clock / power samples (amd-smi) beside tools/clock_probe.py's sustained launches
#   bash tools/clock_probe.sh <out_dir> [probe args...]
set -u
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
timeout -k 10 120 python tools/clock_probe.py "$@" > "$OUT/probe.jsonl" 2> "$OUT/probe.err" &
P=$!
while kill -0 $P 2>/dev/null; do
  echo "=== abs=$(date +%s.%N)" >> "$OUT/smi.txt"
  timeout 5 amd-smi metric -g 0 --clock --power --temperature >> "$OUT/smi.txt" 2>&1 || true
  sleep 0.2
done
wait $P
rc=$?
echo "probe rc=$rc"
tail -3 "$OUT/probe.err"
exit $rc
