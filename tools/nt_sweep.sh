# forward store/load cache-policy variants across graphs (development helper)
mkdir -p gpurun_out
for cfg in "reddit 32 local" "products 8 staged" "products 32 staged"; do
    set -- $cfg
    for v in base ${VARIANTS:-}; do
        lib=""; [ "$v" != base ] && lib=tools/variants/lib_$v.so
        MAXK_LIB=$lib timeout -k 10 300 python bench.py --graph $1 --k $2 --bwd-algo $3 --no-cpu-baseline --no-vendor --steps 10 > gpurun_out/nt.json 2> gpurun_out/nt.err || { tail -5 gpurun_out/nt.err; exit 1; }
        python -c "import json;d=json.load(open('gpurun_out/nt.json'));print('$1 k=$2 $v', d['ms_per_step'], 'fwd', d.get('fwd_ms'), 'bwd', d.get('bwd_ms'))"
    done
done
