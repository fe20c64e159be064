#!/bin/bash
# round 4 closing record: whole GPU suite + smoke, every bench op, the default headline line with its
# kernel stats, and counter passes for the ops that changed late.   bash tools/gpu/gpu_r04final.sh <tag>
set -u
TAG=${1:-final2}
OUT=gpurun_out/r04$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest.txt" 2>&1
rc=$?
tail -2 "$OUT/pytest.txt"
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || exit 1
bash tools/bench_ops.sh r04$TAG gauss5 gauss3 box3 median5 median3 bilateral noise_gaussian noise_sap \
  noise_poisson wavelet_haar3 wavelet_bior15 wavelet_bior15_f64 gauss5_blob quant7 cfg2 cfg3 cfg4 cfg5 \
  jpeg_decode detect_e2e || exit 1
timeout -k 10 300 python bench.py > "$OUT/default.json" 2> "$OUT/default.err" || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/ks_default" -o k --output-format csv \
    -- python3 bench.py --no-cpu > "$OUT/ks_default.json" 2>&1 || exit 1
bash tools/pmc_r04.sh r04$TAG/pmc wavelet_bior15 wavelet_haar3 wavelet_bior15_f64 cfg5 || exit 1
python3 -c "
import json; d=json.load(open('$OUT/default.json')); r=d['roofline']
print('headline', d['value'], 'ms/step', d['ms_per_step'], 'kern', r['kernel_ms_avg'], 'frac', r['frac'], d['copy_ceiling']['by_policy'])"
echo ok
