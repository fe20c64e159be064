#!/bin/bash
# round 5: pitched-tile band height x cache policy (interleaved A/B)
set -u
OUT=${1:-r05b}
bash tools/ab_knobs.sh "$OUT" gauss5 2 product "ntp1s:IDN_STENCIL_NTP=1,IDN_STENCIL_NTS=1" \
  "nb8:X=0@tnb8" "nb8s:IDN_STENCIL_NTP=1,IDN_STENCIL_NTS=1@tnb8" \
  "nb10s:IDN_STENCIL_NTP=1,IDN_STENCIL_NTS=1@tnb10" \
  "nb12:X=0@tnb12" "nb12s:IDN_STENCIL_NTP=1,IDN_STENCIL_NTS=1@tnb12" \
  "nb16s:IDN_STENCIL_NTP=1,IDN_STENCIL_NTS=1@tnb16" \
  "id12s:IDN_STENCIL_IDENT=1,IDN_STENCIL_NTP=1,IDN_STENCIL_NTS=1@tnb12" \
  "nb12nts:IDN_STENCIL_NTS=1@tnb12" || exit 1
