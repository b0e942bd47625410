# LOCAL backward parity subset + Reddit bench (LOCAL and AUTO); development helper
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -k "local or edge_cases or golden or backward" > gpurun_out/lc_tests.log 2>&1; rc=$?; tail -3 gpurun_out/lc_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --bwd-algo local --no-cpu-baseline --steps 10 > gpurun_out/lc_local.json 2> gpurun_out/lc_local.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/lc_local.json'));print('local', d['ms_per_step'], d.get('bwd_ms'), d.get('fwd_ms'))"
