#!/bin/bash
# round 6: the fp32 paired Haar-3 synthesis (wl_h3_synth) -- wavelet / config tests, then A/B of
# the op against the round-4 synthesis (tuning build, IDN_WAVELET_H3S=0) and a kernel trace
set -u
OUT=gpurun_out/${1:-r06b}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_wavelet_gpu.py tests/test_configs_gpu.py -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.txt" 2>&1
rc=$?; tail -3 "$OUT/pytest.txt"; [ $rc = 0 ] || exit $rc
for rep in 1 2; do
  for v in 1 0; do
    IDN_WAVELET_H3S=$v timeout -k 10 120 python bench.py --lib tuning --op wavelet_haar3 --no-cpu \
      --no-copy --steps 20 --warmup 3 > "$OUT/h3s$v.$rep.json" || exit 1
    python3 -c "import json,sys; print(sys.argv[1], json.load(open(sys.argv[2]))['ms_per_step'])" h3s$v "$OUT/h3s$v.$rep.json"
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$(pwd)/$OUT/ks" -o k --output-format csv \
  -- python3 bench.py --op wavelet_haar3 --no-cpu --no-copy --steps 10 --warmup 2 > "$OUT/ks.log" 2>&1 || exit 1
echo ok
