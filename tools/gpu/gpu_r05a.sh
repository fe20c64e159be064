#!/bin/bash
# round 5: pitched-tile stencil -- filter parity, then an interleaved A/B of forms and policies
set -u
OUT=gpurun_out/${1:-r05a}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_filters_gpu.py -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider -k "stencil or gaussian or box or generic" \
    > "$OUT/pytest.txt" 2>&1
rc=$?
tail -3 "$OUT/pytest.txt"
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py > "$OUT/default.json" 2> "$OUT/default.err" || exit 1
cat "$OUT/default.json"
bash tools/ab_knobs.sh "${1:-r05a}/ab" gauss5 2 product "flat:IDN_STENCIL_FORM=0" \
  "ntp1:IDN_STENCIL_NTP=1" "ntp1s:IDN_STENCIL_NTP=1,IDN_STENCIL_NTS=1" \
  "ntp2s:IDN_STENCIL_NTP=2,IDN_STENCIL_NTS=1" "ident:IDN_STENCIL_IDENT=1" \
  "ident_ntp1s:IDN_STENCIL_IDENT=1,IDN_STENCIL_NTP=1,IDN_STENCIL_NTS=1" || exit 1
