# LOCAL backward tuning sweep (development helper): prints ms/step and bwd ms per variant
mkdir -p gpurun_out
one() {  # one <label> <env...>
    local label=$1; shift
    env "$@" timeout -k 10 300 python bench.py --bwd-algo local --no-cpu-baseline --steps 10 > gpurun_out/sw.json 2> gpurun_out/sw.err || { tail -5 gpurun_out/sw.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/sw.json'));print('$label', d['ms_per_step'], d.get('bwd_ms'))"
}
one base MAXK_X=0
one R32 MAXK_LIB=tools/variants/libR32.so
one w8 MAXK_LOCAL_WAVES_PER_CU=8
one w12 MAXK_LOCAL_WAVES_PER_CU=12
one w24 MAXK_LOCAL_WAVES_PER_CU=24
one b16M MAXK_LOCAL_BAND_BYTES=16777216
one b64M MAXK_LOCAL_BAND_BYTES=67108864
one lds8k MAXK_LOCAL_WAVE_LDS=8192
one lds14k MAXK_LOCAL_WAVE_LDS=14336
