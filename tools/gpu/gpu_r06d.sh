#!/bin/bash
# round 6: Haar-3 two-read pipeline -- tests, op time, kernel trace, SQ counters of the kernels
set -u
OUT=gpurun_out/${1:-r06d}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_wavelet_gpu.py tests/test_configs_gpu.py -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.txt" 2>&1
rc=$?; tail -3 "$OUT/pytest.txt"; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python bench.py --op wavelet_haar3 --no-cpu --no-copy --steps 20 --warmup 3 > "$OUT/h3.json" || exit 1
python3 -c "import json,sys; print('h3', json.load(open(sys.argv[1]))['ms_per_step'])" "$OUT/h3.json"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$(pwd)/$OUT/ks" -o k --output-format csv \
  -- python3 bench.py --op wavelet_haar3 --no-cpu --no-copy --steps 10 --warmup 2 > "$OUT/ks.log" 2>&1 || exit 1
S1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
S2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for pass in sq1 sq2; do
  C=$S1; [ $pass = sq2 ] && C=$S2
  timeout -s KILL 90 rocprofv3 --pmc $C -d "$(pwd)/$OUT/$pass" -o pmc --output-format csv \
    -- python3 bench.py --op wavelet_haar3 --no-cpu --no-copy --steps 3 --warmup 1 --settle-s 0 > "$OUT/$pass.log" 2>&1 || exit 1
done
echo ok
