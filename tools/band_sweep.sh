mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -q -m gpu -k "local or edge_cases or golden" > gpurun_out/band_tests.log 2>&1; rc=$?; tail -3 gpurun_out/band_tests.log; [ $rc -le 1 ] || exit $rc
for b in 1099511627776 67108864 33554432 16777216 8388608; do
  MAXK_LOCAL_BAND_BYTES=$b timeout -k 10 300 python bench.py --bwd-algo local --no-cpu-baseline --steps 10 > gpurun_out/band_$b.json 2> gpurun_out/band_$b.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/band_$b.json'));print($b, d['ms_per_step'], d.get('bwd_ms'), d.get('fwd_ms'))"
done
