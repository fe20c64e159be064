#!/bin/bash
# round 6: the whole GPU suite (EXIF orientation, restart-interval zero fill) and smoke
set -u
OUT=gpurun_out/${1:-r06a}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest.txt" 2>&1
rc=$?
tail -5 "$OUT/pytest.txt"
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || exit 1
tail -1 "$OUT/smoke.txt"
