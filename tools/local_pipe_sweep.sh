# LOCAL backward variants on Reddit / proteins-like shapes (development helper)
mkdir -p gpurun_out
for cfg in ${CFGS:-"reddit 32" "reddit 64" "reddit 16"}; do
    set -- $cfg
    for v in base ${VARIANTS:-}; do
        lib=""; [ "$v" != base ] && lib=tools/variants/lib_$v.so
        MAXK_LIB=$lib timeout -k 10 300 python bench.py --graph $1 --k $2 --bwd-algo local --no-cpu-baseline --no-vendor --steps 10 > gpurun_out/lp.json 2> gpurun_out/lp.err || { tail -5 gpurun_out/lp.err; exit 1; }
        python -c "import json;d=json.load(open('gpurun_out/lp.json'));print('$1 k=$2 $v', d['ms_per_step'], 'fwd', d.get('fwd_ms'), 'bwd', d.get('bwd_ms'))"
    done
done
