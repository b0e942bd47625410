# BASELINE configs 3 and 5 on one GPU (development helper): products k sweep, proteins R=8 fused forward
mkdir -p gpurun_out/configs
timeout -k 10 300 python bench.py --graph proteins --relations 8 --steps 10 > gpurun_out/configs/proteins_r8.json 2> gpurun_out/configs/proteins_r8.err || exit $?
cat gpurun_out/configs/proteins_r8.json
for k in 8 16 32 64; do
  timeout -k 10 400 python bench.py --graph products --k $k --no-cpu-baseline --steps 10 > gpurun_out/configs/products_k$k.json 2> gpurun_out/configs/products_k$k.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/configs/products_k$k.json'));print('products k=$k', d['ms_per_step'], d['value'], d['fwd_ms'], d['bwd_ms'], d['config']['bwd_algo'], d.get('topk_ms'), d.get('scatter_ms'))"
done
