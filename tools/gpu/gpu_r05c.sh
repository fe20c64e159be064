#!/bin/bash
# round 5: pitched-tile band height 8-10 x halo load policy (interleaved A/B)
set -u
OUT=${1:-r05c}
S="IDN_STENCIL_NTS=1"
bash tools/ab_knobs.sh "$OUT" gauss5 2 product \
  "nb8s:IDN_STENCIL_NTP=1,$S@tnb8" "nb8p3:IDN_STENCIL_NTP=3,$S@tnb8" "nb8p4:IDN_STENCIL_NTP=4,$S@tnb8" \
  "nb9s:IDN_STENCIL_NTP=1,$S@tnb9" "nb9p3:IDN_STENCIL_NTP=3,$S@tnb9" \
  "nb10s:IDN_STENCIL_NTP=1,$S@tnb10" "nb10p3:IDN_STENCIL_NTP=3,$S@tnb10" \
  "nb10p4:IDN_STENCIL_NTP=4,$S@tnb10" "id8s:IDN_STENCIL_IDENT=1,IDN_STENCIL_NTP=1,$S@tnb8" \
  "id10s:IDN_STENCIL_IDENT=1,IDN_STENCIL_NTP=1,$S@tnb10" || exit 1
