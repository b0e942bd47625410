#!/bin/bash
# Development: build libmaxk_spgemm variants of maxk_spgemm.hip with extra flags,
# linked with the product build's topk / plan objects (run build() first).
#   tools/build_fwd_variants.sh name:"-DFLAG=1 ..." name2:"..."  -> tools/variants/lib_<name>.so
# The ablation switches (FWD_ABLATE, ...) come from tools/ablate/product_ablations.patch,
# applied to a copy of the product source (see tools/build_variant.sh).
cd "$(dirname "$0")/.." || exit 2
mkdir -p tools/variants/src
cp spgemm_new_amd/csrc/maxk_spgemm.hip tools/variants/src/maxk_spgemm.hip
patch -s tools/variants/src/maxk_spgemm.hip < tools/ablate/product_ablations.patch || exit 2
O=spgemm_new_amd/lib/obj
for spec in "$@"; do
    name=${spec%%:*}; flags=${spec#*:}
    ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -I include \
        -I spgemm_new_amd/csrc $flags \
        tools/variants/src/maxk_spgemm.hip -o tools/variants/$name.o &&
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/variants/lib_$name.so \
        tools/variants/$name.o $O/maxk_topk.hip.o $O/maxk_plan.hip.o && echo "built $name" ) &
done
wait
