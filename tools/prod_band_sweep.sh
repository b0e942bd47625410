# LOCAL on products with larger source bands (development helper)
mkdir -p gpurun_out
for k in 8 32; do
  for b in 33554432 134217728 268435456; do
    MAXK_LOCAL_BAND_BYTES=$b timeout -k 10 300 python bench.py --graph products --k $k --bwd-algo local --no-cpu-baseline --no-vendor --steps 5 > gpurun_out/pb.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/pb.json'));print('k=$k band=$b', 'bwd', d['bwd_ms'])"
  done
done
