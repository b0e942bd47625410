# ATOMIC backward variants across graphs and k (development helper)
mkdir -p gpurun_out
for cfg in ${CFGS:-"reddit 32" "products 8" "products 16" "products 32"}; do
    set -- $cfg
    for v in base ${VARIANTS:-}; do
        lib=""; [ "$v" != base ] && lib=tools/variants/lib_$v.so
        MAXK_LIB=$lib timeout -k 10 300 python bench.py --graph $1 --k $2 --bwd-algo ${ALGO:-atomic} --no-cpu-baseline --no-vendor --steps 10 > gpurun_out/as.json 2> gpurun_out/as.err || { tail -5 gpurun_out/as.err; exit 1; }
        python -c "import json;d=json.load(open('gpurun_out/as.json'));print('$1 k=$2 $v', d['ms_per_step'], 'fwd', d.get('fwd_ms'), 'bwd', d.get('bwd_ms'))"
    done
done
