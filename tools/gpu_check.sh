#!/bin/bash
# One GPU-box session: parity tests, smoke, bench.  Stops at the first step
# that crashes or times out (exit codes other than 0 / 1); test failures (1)
# are reported but later steps still run.
# usage: tools/gpu_check.sh [pytest-args...]   (env: BENCH_ARGS, SKIP_TESTS, SKIP_BENCH)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
ok_or_fail() {  # continue only on 0 / 1
    local rc=$1 what=$2
    echo "[gpu_check] $what rc=$rc"
    if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
        echo "[gpu_check] stopping after $what (rc=$rc)"; exit "$rc"
    fi
}
if [ -z "$SKIP_TESTS" ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread "$@" \
        > gpurun_out/pytest_gpu.log 2>&1
    ok_or_fail $? pytest_gpu
    tail -5 gpurun_out/pytest_gpu.log
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
    ok_or_fail $? smoke
    tail -2 gpurun_out/smoke.log
fi
if [ -z "$SKIP_BENCH" ]; then
    timeout -k 10 600 python bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err
    ok_or_fail $? bench
    cat gpurun_out/bench.json
fi
exit 0
