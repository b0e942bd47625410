"""bench.py's output contract (the driver parses its last stdout line): one JSON
object with the metric, whole-job value, timing fields, roofline and
cpu_baseline objects.  Runs a small configuration as a subprocess (GPU)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["--partitioned"], ["--graph", "proteins", "--relations", "4"]])
def test_bench_json_line(extra):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--graph", "flickr", "--h", "64",
           "--k", "16", "--steps", "2", "--warmup", "1", "--cpu-seconds", "1", "--no-vendor"] + extra
    if "--relations" in extra:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
               "--k", "32"] + extra
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    line = out.stdout.strip().splitlines()[-1]
    d = json.loads(line)
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
                "roofline"):
        assert key in d, key
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["value"] > 0
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["peak"] == 8000.0 and 0 < r["frac"] < 1.5
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    if not extra:
        cb = d["cpu_baseline"]
        assert cb["kind"] == "reference" and cb["value"] > 0 and cb["cores"] >= 1
        assert "sample" in cb and cb["mean_form_fwd_ms_sample"] > 0
        assert cb["ms_per_step_full_graph"] > 0 and 0 < cb["edge_fraction"] <= 1
        bc = d["bwd_check"]   # the timed dx vs STAGED, and the adjoint identity
        assert bc["max_rel_diff"] <= 1e-4 and bc["adjoint_rel_err"] <= 1e-6


@pytest.mark.gpu
def test_bench_two_ranks_rehearsal():
    """The N>1 bench path (torch.distributed.run, row partition, halo exchange,
    max-over-ranks timing) end to end with 2 ranks on one GPU; gloo stands in
    for RCCL (BENCH_BACKEND=gloo), so only the logic is exercised here."""
    env = dict(os.environ, BENCH_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29613", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--graph", "flickr", "--h", "64",
           "--k", "16", "--overlap", "on"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads(out.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "rowpart2"
    assert d["value"] > 0 and d["roofline"]["achieved"] > 0
    assert d["config"]["halo_nodes_rank0"] > 0 and d["config"]["overlap"] is True
    assert d["config"]["halo_mode"] in ("records", "allgather")
    assert d["config"]["halo_bytes_rank0"]["reverse_bwd"] > 0


@pytest.mark.gpu
def test_bench_two_ranks_multi_relation_rehearsal():
    """Config 5's N>1 path (bench.py --relations R under torch.distributed.run):
    partitioned fused multi-relation forward + backward, 2 ranks on one GPU, gloo."""
    env = dict(os.environ, BENCH_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29617", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--graph", "flickr", "--h", "64",
           "--k", "16", "--relations", "8"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads(out.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "rowpart2"
    assert d["config"]["relations"] == 8 and d["value"] > 0 and d["bwd_multi_ms"] > 0


@pytest.mark.gpu
def test_bench_launches_its_own_ranks():
    """`python bench.py --gpus 2` with no outside launcher: the
    parent makes no GPU call, starts 2 ranks itself (gloo stands in for RCCL, both
    ranks on the one GPU) and relays rank 0's line, which reports n_gpus 2, the
    row partition and the per-exchange wire times."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK",
                                                            "MASTER_PORT")}
    env["BENCH_BACKEND"] = "gloo"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--graph", "flickr", "--h", "64", "--k", "16"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = out.stdout.strip().splitlines()
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "rowpart2"
    ex = d["exchange_ms_max_over_ranks"]
    assert ex["bwd_a2a_ms"] > 0 and ("fwd_a2a_ms" in ex or "fwd_allgather_ms" in ex)


@pytest.mark.gpu
def test_bench_n2_reports_multi_gpu_configs():
    """one `bench.py --gpus N` launch (what the driver's scaling
    runs call) also measures BASELINE config 4 (products k=32) and config 5
    (proteins R=8) row-partitioned, in the `configs` of rank 0's line.  2 ranks on
    the one GPU, gloo standing in for RCCL (host-staged exchanges: plumbing only)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK",
                                                            "MASTER_PORT")}
    env["BENCH_BACKEND"] = "gloo"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--config-steps", "2"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=900, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads(out.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "rowpart2"
    c = d["configs"]
    p, q = c["products_k32_rowpart2"], c["proteins_r8_rowpart2"]
    for e in (p, q):
        assert e["n_gpus"] == 2 and e["parallelism"] == "rowpart2" and e["ms_per_step"] > 0
        assert e["fwd_ms"]["median_max_over_ranks"] > 0 and e["bwd_ms"]["median_max_over_ranks"] > 0
        assert e["check"]["adjoint_rel_err"] < 1e-6
    assert p["baseline_config"] == 4 and p["num_nodes"] == 2449029
    assert p["halo_mode"] in ("records", "allgather") and p["halo_bytes_rank0"]["reverse_bwd"] > 0
    assert p["exchange_ms_max_over_ranks"]["bwd_a2a_ms"] > 0
    assert q["baseline_config"] == 5 and q["relations"] == 8 and q["num_nodes"] == 132534


@pytest.mark.gpu
def test_bench_more_gpus_than_visible_fails():
    """--gpus 9 on a one-GPU box (RCCL: one GPU per rank) exits non-zero, prints no line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK",
                                                            "BENCH_BACKEND")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "9"],
                         cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode != 0 and out.stdout.strip() == ""
