set -u
mkdir -p gpurun_out/jchunk
for c in 2048 4096 8192 16384; do
  IDN_JPEG_CHUNK=$c timeout -k 10 200 python bench.py --op jpeg_decode --no-copy --no-cpu --steps 10 --warmup 2 > gpurun_out/jchunk/b_$c.json 2>/dev/null || exit 1
  echo $c $(python -c "import json;d=json.load(open('gpurun_out/jchunk/b_$c.json'));print(d['ms_per_step'])")
done
