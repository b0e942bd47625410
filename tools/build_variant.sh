#!/bin/bash
# Build a development variant of libmaxk_spgemm.so with extra compile flags:
#   tools/build_variant.sh <name> [-DFLAG ...]  ->  tools/variants/lib_<name>.so
# (load it with MAXK_LIB=$PWD/tools/variants/lib_<name>.so; development only)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p tools/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -I include "$@" \
    -o tools/variants/lib_$name.so spgemm_new_amd/csrc/maxk_spgemm.hip \
    spgemm_new_amd/csrc/maxk_topk.hip spgemm_new_amd/csrc/maxk_plan.hip
echo "built tools/variants/lib_$name.so"
