# CBSR entry order vs kernel time (development helper)
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_topk.py -q -x -p no:cacheprovider > gpurun_out/t.log 2>&1 || { tail -5 gpurun_out/t.log; exit 1; }
for o in column lane value; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --cbsr-order $o > gpurun_out/o.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/o.json'));print('$o', d['ms_per_step'], 'fwd', d['fwd_ms'], 'bwd', d['bwd_ms'])"
done
