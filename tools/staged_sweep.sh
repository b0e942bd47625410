# STAGED store-form variant on Reddit and products k=32 (development helper)
mkdir -p gpurun_out
for g in reddit products; do
  for lib in "" tools/variants/lib_STAGED_PLAIN_STORE.so; do
    MAXK_LIB=$lib timeout -k 10 300 python bench.py --graph $g --bwd-algo staged --no-cpu-baseline --steps 10 > gpurun_out/s.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s.json'));print('$g', '${lib:-base}', d['ms_per_step'], 'fwd', d['fwd_ms'], 'bwd', d['bwd_ms'])"
  done
done
