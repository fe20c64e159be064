#!/bin/bash
# round 4 checkpoint: whole GPU suite, smoke(), default bench line.   bash tools/gpu/gpu_r04s.sh
set -u
OUT=gpurun_out/r04s
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest.txt" 2>&1
rc=$?
tail -3 "$OUT/pytest.txt"
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
tail -2 "$OUT/smoke.txt"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']
print('headline ms/step', d['ms_per_step'], 'kern', r['kernel_ms_avg'], 'frac', r['frac'], 'copy default', d['copy_ceiling']['by_policy'])"
echo ok
