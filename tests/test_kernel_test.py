"""The maxk_kernel_test executable (kernels/main.cu on the C ABI)."""
import os
import subprocess

import numpy as np
import pytest

from spgemm_new_amd.graphs import small_csr, write_csr

HERE = os.path.dirname(os.path.abspath(__file__))
BIN = os.path.join(HERE, "..", "spgemm_new_amd", "lib", "maxk_kernel_test")


def test_harness_built():
    """build() produced the harness; --help needs no GPU."""
    assert os.path.exists(BIN), "run __graft_entry__.build() first"
    r = subprocess.run([BIN, "--help"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "usage" in r.stdout


@pytest.mark.gpu
def test_harness_runs_and_validates(tmp_path):
    """main.cu's output lines for k = 16 / 32 / 64, every backward algorithm (TILE
    at k = 32 / 64, its plan built by maxk_tile_plan_build; APPEND with node and
    edge selectors, its plan built by maxk_append_plan_build),
    and the --check validations (forward vs dense SpMM, backward algorithms
    against each other) on two small graphs read from raw int32 files."""
    for name, seed in (("g1", 3), ("g2", 4)):
        indptr, indices = small_csr(2000, seed=seed)
        write_csr(str(tmp_path / name), indptr, indices)
    r = subprocess.run([BIN, "--dir", str(tmp_path), "--check"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.splitlines()
    times = {}
    for ln in lines:
        f = ln.split()
        if len(f) == 6 and "/" in f[0]:
            times[(f[1], int(f[3]), f[4])] = float(f[5])
    for g in ("g1", "g2"):
        assert (g, 16, "dense_spmm") in times
        for k in (16, 32, 64):
            algos = ["maxk_backward_atomic", "maxk_backward_staged", "maxk_backward_staged_edge",
                     "maxk_backward_append", "maxk_backward_append_edge", "maxk_backward_local"]
            if k in (32, 64):
                algos.append("maxk_backward_tile")   # the TILE plan through the C ABI
            fwds = ["maxk"] + (["maxk_blocked4"] if k >= 32 else [])   # column-blocked forward
            for kern in fwds + ["maxk_backward"] + algos:
                assert times[(g, k, kern)] > 0, (g, k, kern)
            assert times[(g, k, "maxk_backward")] == min(times[(g, k, a)] for a in algos)
    checks = [ln for ln in lines if "validation" in ln]
    # per graph: k=16 fwd + staged + staged_edge + append + append_edge + local;
    # k=32 and k=64 also tile and the blocked forward
    assert len(checks) == 2 * (6 + 8 + 8), checks
    assert all("validation pass!" in ln for ln in checks), checks
    assert sum("backward tile vs atomic" in ln for ln in checks) == 4
    assert sum("forward blocked4 vs plain" in ln for ln in checks) == 4
    assert sum("backward append_edge vs atomic" in ln for ln in checks) == 6
    assert np.isfinite(list(times.values())).all()
