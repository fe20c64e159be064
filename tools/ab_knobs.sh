#!/bin/bash
# Same-run A/B of tuning knobs on one bench op, interleaved:
#   bash tools/ab_knobs.sh <out_dir> <op> <reps> <spec> ...
# spec = "product" (the product library) or "label:KNOB=v,KNOB=v[@variant]" (the tuning library
# with those knobs set; @variant: ab/<variant>.so, from tools/build_variant.py --base tuning,
# stands in for the tuning library).  Each run is a full bench line (warmup, 0.5 s settle, 100
# timed steps, no CPU leg).
set -u
OUT=gpurun_out/$1; OP=$2; REPS=$3; shift 3
mkdir -p "$OUT"
TL=image-denoising_amd/idn/libidn_hip_tuning.so
cp $TL "$OUT/.tuning_intree.so"
trap 'cp "$OUT/.tuning_intree.so" $TL; rm -f "$OUT/.tuning_intree.so"' EXIT
for rep in $(seq 1 "$REPS"); do
  for spec in "$@"; do
    label=${spec%%:*}
    if [ "$spec" = "product" ]; then
      timeout -k 10 120 python bench.py --op "$OP" --no-cpu --no-copy >> "$OUT/$label.jsonl" 2>> "$OUT/ab.err" || exit 1
    else
      body=${spec#*:}
      if [ "${body#*@}" != "$body" ]; then cp "ab/${body#*@}.so" $TL || exit 1; body=${body%@*};
      else cp "$OUT/.tuning_intree.so" $TL; fi
      env $(echo "$body" | tr ',' ' ') timeout -k 10 120 python bench.py --op "$OP" --lib tuning \
        --no-cpu --no-copy >> "$OUT/$label.jsonl" 2>> "$OUT/ab.err" || exit 1
    fi
  done
done
for spec in "$@"; do
  label=${spec%%:*}
  python3 - "$OUT/$label.jsonl" "$label" <<'PY'
import json, sys
recs = [json.loads(l) for l in open(sys.argv[1]) if l.strip()]
ms = [r["roofline"]["kernel_ms_avg"] for r in recs]
gb = [r["roofline"]["achieved"] for r in recs]
print(f"{sys.argv[2]:>14}: kernel_ms {' '.join(f'{m:.5f}' for m in ms)}  GB/s {' '.join(f'{g:.0f}' for g in gb)}")
PY
done
