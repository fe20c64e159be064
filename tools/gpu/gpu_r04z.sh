#!/bin/bash
# round-4 last check of HEAD: the whole GPU suite, smoke, the default bench line
set -u
OUT=gpurun_out/${1:-r04z}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest.txt" 2>&1
rc=$?
tail -2 "$OUT/pytest.txt"
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || exit 1
tail -1 "$OUT/smoke.txt"
timeout -k 10 300 python bench.py > "$OUT/default.json" 2> "$OUT/default.err" || exit 1
cat "$OUT/default.json"
