# forward variant sweep (development helper)
mkdir -p gpurun_out
one() {
    local label=$1; shift
    env "$@" timeout -k 10 300 python bench.py --bwd-algo local --no-cpu-baseline --steps 10 > gpurun_out/sw.json 2> gpurun_out/sw.err || { tail -5 gpurun_out/sw.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/sw.json'));print('$label', d['ms_per_step'], 'fwd', d.get('fwd_ms'), 'bwd', d.get('bwd_ms'))"
}
one base MAXK_X=0
for v in ${VARIANTS:-}; do one $v MAXK_LIB=tools/variants/lib_$v.so; done
