#!/bin/bash
# rocprofv3 passes over a short bench run (kernel trace + stats, then one PMC
# group per pass; counters never combined with runtime/sys tracing).
# usage: tools/profile.sh <tag> [bench args...]
# output: gpurun_out/prof_<tag>/{trace,pmc_*}/...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
tag=${1:-run}; shift
out=gpurun_out/prof_$tag
mkdir -p "$out"
BENCH=(python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-vendor --no-configs "$@")
run() {  # run <name> <rocprof args...>
    local name=$1; shift
    timeout -k 10 600 rocprofv3 "$@" -d "$out/$name" -o "$name" --output-format csv -T \
        -- "${BENCH[@]}" > "$out/$name.log" 2>&1
    local rc=$?
    echo "[profile] $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -20 "$out/$name.log"; exit $rc; fi
}
run trace --kernel-trace --stats
PMCS=("SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
        "SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
        "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum")
[ -n "$PMC_GROUPS" ] && IFS=';' read -r -a PMCS <<< "$PMC_GROUPS"   # ';'-separated groups
[ -n "$NO_PMC" ] && PMCS=()
for grp in "${PMCS[@]}"; do
    name=pmc_$(echo "$grp" | tr ' ' '_' | cut -c1-40)
    run "$name" --kernel-trace --pmc $grp
done
exit 0
