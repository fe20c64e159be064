#!/bin/bash
# round 5 checkpoint: the whole GPU suite, smoke, the default bench line, its kernel-trace stats,
# and the counter passes of the three u8 stencils
set -u
OUT=gpurun_out/${1:-r05f}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest.txt" 2>&1
rc=$?
tail -2 "$OUT/pytest.txt"
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || exit 1
tail -1 "$OUT/smoke.txt"
timeout -k 10 300 python bench.py > "$OUT/default.json" 2> "$OUT/default.err" || exit 1
cat "$OUT/default.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$(pwd)/$OUT/ks" -o k --output-format csv \
  -- python3 bench.py --no-cpu > "$OUT/ks.log" 2>&1 || exit 1
bash tools/pmc_r04.sh "${1:-r05f}/pmc" gauss5 gauss3 box3 || exit 1
