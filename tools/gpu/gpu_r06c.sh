#!/bin/bash
# round 6: the two-read Haar-3 pipeline (wl_h3_window / stats / sigma / synth) -- wavelet and config
# tests, A/B of the op against the round-5 passes (tuning build, IDN_WAVELET_H3=0), kernel trace
set -u
OUT=gpurun_out/${1:-r06c}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_wavelet_gpu.py tests/test_configs_gpu.py -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.txt" 2>&1
rc=$?; tail -30 "$OUT/pytest.txt"; [ $rc = 0 ] || exit $rc
for rep in 1 2; do
  for v in 1 0; do
    IDN_WAVELET_H3=$v timeout -k 10 120 python bench.py --lib tuning --op wavelet_haar3 --no-cpu \
      --no-copy --steps 20 --warmup 3 > "$OUT/h3_$v.$rep.json" || exit 1
    python3 -c "import json,sys; print(sys.argv[1], json.load(open(sys.argv[2]))['ms_per_step'])" h3_$v "$OUT/h3_$v.$rep.json"
  done
done
timeout -k 10 120 python bench.py --op cfg5 --no-cpu --no-copy --steps 20 --warmup 3 > "$OUT/cfg5.json" || exit 1
python3 -c "import json,sys; print('cfg5', json.load(open(sys.argv[1]))['ms_per_step'])" "$OUT/cfg5.json"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$(pwd)/$OUT/ks" -o k --output-format csv \
  -- python3 bench.py --op wavelet_haar3 --no-cpu --no-copy --steps 10 --warmup 2 > "$OUT/ks.log" 2>&1 || exit 1
echo ok
