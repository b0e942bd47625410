#!/bin/bash
# Build a development variant of libmaxk_spgemm.so with extra compile flags:
#   tools/build_variant.sh <name> [-DFLAG ...]  ->  tools/variants/lib_<name>.so
# (load it with MAXK_LIB=$PWD/tools/variants/lib_<name>.so; development only)
# The timing-ablation switches (FWD_ABLATE, LOCAL_ABLATE, TILE_ABLATE: results wrong)
# are not in the product source since round 6: they live in
# tools/ablate/product_ablations.patch, applied here to a copy of maxk_spgemm.hip.
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p tools/variants/src
cp spgemm_new_amd/csrc/maxk_spgemm.hip tools/variants/src/maxk_spgemm.hip
patch -s tools/variants/src/maxk_spgemm.hip < tools/ablate/product_ablations.patch
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -I include \
    -I spgemm_new_amd/csrc "$@" \
    -o tools/variants/lib_$name.so tools/variants/src/maxk_spgemm.hip \
    spgemm_new_amd/csrc/maxk_topk.hip spgemm_new_amd/csrc/maxk_plan.hip
echo "built tools/variants/lib_$name.so"
