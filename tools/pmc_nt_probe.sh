set -e
mkdir -p gpurun_out/pmc_nt
for nt in 0 1 3; do
  IDN_STENCIL_IDENT=1 IDN_STENCIL_NT=$nt timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_nt/f$nt -o pmc --output-format csv -- python3 bench.py --no-cpu --no-copy --steps 5 --warmup 2 --settle-s 0 > gpurun_out/pmc_nt/f$nt.log 2>&1
  echo "nt=$nt ok"
done
