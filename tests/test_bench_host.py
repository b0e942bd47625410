"""Host logic of bench.py (no GPU): roofline traffic composed from the committed
per-kernel PMC bytes, keyed to the kernel sources it was measured on; the
issue-rate roofline from SQ counters; the workload key."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

KERN = {"bwd_local_kernel": 2.0e9, "fwd_panel_kernel": 20.0e9, "carry_fixup_owner_kernel": 1.0e8,
        "bwd_tile_kernel": 2.3e9, "tile_combine_kernel": 9.0e7}


def _index(tmp_path, monkeypatch, sha):
    idx = {"reddit_h256_k32_local": {"profile": "r9_test", "source_sha": sha, "kernels": KERN},
           "reddit_h256_k32_tile": {
               "profile": "r9_test", "source_sha": sha, "kernels": KERN,
               "issue": {"bwd_tile_kernel": {"avg_ms": 3.0, "GRBM_GUI_ACTIVE": 8 * 7.2e6,
                                             "SQ_INSTS_SALU": 0.5 * 256 * 7.2e6,
                                             "SQ_INSTS_VALU": 0.25 * 2 * 256 * 7.2e6}}}}
    p = tmp_path / "pmc_traffic.json"
    p.write_text(json.dumps(idx))
    monkeypatch.setattr(bench, "PMC_INDEX", str(p))


def test_pmc_traffic_composition(tmp_path, monkeypatch):
    _index(tmp_path, monkeypatch, bench.kernel_source_sha())
    t, src, stale = bench.pmc_traffic("reddit_h256_k32_local", "sspmm_backward", "local", 8)
    assert t == int(KERN["bwd_local_kernel"] * 8) and stale is None
    assert src == "profiles/r9_test_summary.json"
    t, _, _ = bench.pmc_traffic("reddit_h256_k32_local", "spgemm_forward", "local", 8)
    assert t == int(KERN["fwd_panel_kernel"] + KERN["carry_fixup_owner_kernel"])
    t, _, _ = bench.pmc_traffic("reddit_h256_k32_tile", "sspmm_backward", "tile", 1)
    assert t == int(KERN["bwd_tile_kernel"] + KERN["tile_combine_kernel"])
    assert bench.pmc_traffic("no_such_workload", "sspmm_backward", "local", 1) == (None, None, None)


def test_stale_profile_is_refused(tmp_path, monkeypatch):
    """A profile taken on other kernel sources is reported as stale, never used."""
    _index(tmp_path, monkeypatch, "0" * 16)
    t, src, stale = bench.pmc_traffic("reddit_h256_k32_tile", "sspmm_backward", "tile", 1)
    assert t is None and src == "profiles/r9_test_summary.json"
    assert stale["profiled_source_sha"] == "0" * 16
    assert stale["current_source_sha"] == bench.kernel_source_sha()
    assert bench.issue_bound("reddit_h256_k32_tile", "bwd_tile_kernel", 3.0, 256) is None


def test_issue_bound(tmp_path, monkeypatch):
    _index(tmp_path, monkeypatch, bench.kernel_source_sha())
    r = bench.issue_bound("reddit_h256_k32_tile", "bwd_tile_kernel", 3.0, 256)
    assert r["busy_frac"]["SQ_INSTS_SALU"] == 0.5 and r["busy_frac"]["SQ_INSTS_VALU"] == 0.25
    assert r["bound"] == "SQ_INSTS_SALU" and r["frac"] == 0.5
    assert abs(r["clock_GHz"] - 2.4) < 1e-9


def test_source_sha_covers_kernels():
    sha = bench.kernel_source_sha()
    assert len(sha) == 16 and all(os.path.exists(os.path.join(ROOT, f)) for f in bench.KERNEL_SOURCES)


def test_committed_profile_index_is_keyed():
    """Every committed profile entry names the kernel sources it measured (a
    missing key reads as stale, so the bench line can never carry an unkeyed
    traffic figure)."""
    idx = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    for name, ent in idx.items():
        assert "profile" in ent and "kernels" in ent, name
        if "source_sha" not in ent:
            t, _, stale = bench.pmc_traffic(name, "sspmm_backward", "tile", 1)
            assert t is None and stale is not None


def test_workload_key():
    class A:
        graph, h, k = "reddit", 256, 32
    assert bench.workload_key(A, "tile") == "reddit_h256_k32_tile"


def test_median():
    assert bench._median([3.0, 1.0, 2.0]) == 2.0
    assert bench._median([4.0, 1.0, 2.0, 3.0]) == 2.5


def test_gpus_beyond_visible_devices_fails_loudly():
    """`bench.py --gpus N` without a launcher starts its own ranks; when N exceeds
    the visible GPUs (none in this container) it exits non-zero before any GPU
    call instead of measuring one GPU and reporting it as N."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "9"],
                         cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode != 0
    assert out.stdout.strip() == ""
    assert "refusing" in out.stderr or "no GPU" in out.stderr


def test_world_size_mismatch_fails_loudly():
    """A launcher that started another number of ranks than --gpus names: refused."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"],
                         cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 6 and out.stdout.strip() == ""


def test_vendor_backward_reference_matches_oracle():
    """bench.vendor_backward_reference (the full-size backward check: A^T by torch,
    torch.sparse.mm, gathered at sel) equals the fp64 oracle on a small graph
    (CPU torch here; rocSPARSE on the GPU), also for a row block (indptr[0] != 0
    views are not used; a rectangular block with more columns than rows is)."""
    import numpy as np
    import torch
    from oracle import oracle as O
    from spgemm_new_amd.graphs import random_cbsr, small_csr
    indptr, indices = small_csr(700, seed=3)
    v, h, k = len(indptr) - 1, 64, 8
    values = np.random.default_rng(1).random(len(indices), dtype=np.float32)
    grad = np.random.default_rng(2).random((v, h), dtype=np.float32)
    _, sel = random_cbsr(v, k, h, seed=4)
    ref = bench.vendor_backward_reference(torch.from_numpy(indptr), torch.from_numpy(indices),
                                          torch.from_numpy(values), torch.from_numpy(grad),
                                          torch.from_numpy(sel))
    want = O.np_backward(indptr, indices, values, grad, sel)
    assert O.parity_error(ref.numpy(), want) <= 1e-4
    # rectangular: the first 300 rows, all 700 columns
    r = 300
    ip = indptr[: r + 1]
    ref = bench.vendor_backward_reference(torch.from_numpy(ip), torch.from_numpy(indices),
                                          torch.from_numpy(values), torch.from_numpy(grad[:r]),
                                          torch.from_numpy(sel), num_cols=v)
    want = O.np_backward(ip, indices[: ip[-1]], values[: ip[-1]], grad[:r], sel)
    assert O.parity_error(ref.numpy(), want) <= 1e-4
