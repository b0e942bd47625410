"""Host logic of bench.py (no GPU): roofline traffic composed from the committed
per-kernel PMC bytes, and the workload key."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_pmc_traffic_composition():
    idx = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    ent = idx["reddit_h256_k32_local"]
    kern = ent["kernels"]
    t, src = bench.pmc_traffic("reddit_h256_k32_local", "sspmm_backward", "local", 8)
    assert t == int(kern["bwd_local_kernel"] * 8)
    assert src == f"profiles/{ent['profile']}_summary.json" and os.path.exists(os.path.join(ROOT, src))
    t, _ = bench.pmc_traffic("reddit_h256_k32_local", "spgemm_forward", "local", 8)
    fix = kern.get("carry_fixup_owner_kernel", kern.get("carry_fixup_kernel", 0.0))
    assert t == int(kern["fwd_panel_kernel"] + fix)
    assert bench.pmc_traffic("no_such_workload", "sspmm_backward", "local", 1) == (None, None)


def test_committed_profile_matches_current_workload():
    """The default bench workload (Reddit h=256 k=32, AUTO -> LOCAL) has a
    committed PMC profile, so its bench line carries a measured traffic."""
    class A:
        graph, h, k = "reddit", 256, 32
    key = bench.workload_key(A, "local")
    assert key == "reddit_h256_k32_local"
    assert bench.pmc_traffic(key, "sspmm_backward", "local", 8)[0] > 0
