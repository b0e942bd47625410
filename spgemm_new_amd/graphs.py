"""Graph inputs: raw CSR files and seeded synthetic graphs.

* ``read_csr`` / ``write_csr`` use the reference's on-disk format: raw
  little-endian int32 ``<g>.indptr`` and ``<g>.indices`` (kernels/data.h:8-24,
  kernels/main.cu:57-58).
* ``synthetic_csr_gpu`` builds Reddit- / ogbn-products-shaped graphs directly in
  HBM (the datasets are not available offline): power-law out-degrees with the
  requested mean, columns uniform without duplicates, sorted per row.  Columns
  (``synthetic_columns``) and edge values (``synthetic_values``) are hashes of
  (seed, edge id), so a rank of the row partition generates only its rows.
* ``small_csr`` builds the small CPU graphs used by the parity tests, with a
  degree mix that exercises degree-0 rows, rows split across panels and the
  reference's 64-nnz chunk boundaries (63/64/65, >200).

The shapes of the benchmark configurations are in ``CONFIGS``.
"""
from __future__ import annotations

import os

import numpy as np
import torch

# name -> (num_rows, num_edges); V from kernels/maxk_kernel.cu:13-16, E public stats.
CONFIGS = {
    "reddit": (232_965, 114_615_892),
    "products": (2_449_029, 123_718_280),
    "proteins": (132_534, 79_122_504),
    "flickr": (89_250, 899_756 + 89_250),  # with self loops (scripts_train/flickr_maxk.sh:15)
}


def read_csr(prefix: str):
    indptr = np.fromfile(prefix + ".indptr", dtype=np.int32)
    indices = np.fromfile(prefix + ".indices", dtype=np.int32)
    return indptr, indices


def write_csr(prefix: str, indptr, indices) -> None:
    os.makedirs(os.path.dirname(prefix) or ".", exist_ok=True)
    np.asarray(indptr, dtype=np.int32).tofile(prefix + ".indptr")
    np.asarray(indices, dtype=np.int32).tofile(prefix + ".indices")


def powerlaw_degrees(num_rows: int, num_edges: int, gen: torch.Generator, device,
                     alpha: float = 2.2, max_factor: float = 64.0) -> torch.Tensor:
    """Integer degrees summing exactly to num_edges, Pareto(alpha)-shaped,
    capped at ~min(num_rows/4, max_factor * mean)."""
    mean = num_edges / num_rows
    # cap well below V so that rejection of duplicate columns converges fast
    cap = int(min(num_rows, max(2.0 * mean + 1, min(num_rows / 4.0, max_factor * mean))))
    if num_edges > cap * num_rows:
        raise ValueError("num_edges too large for the degree cap")
    u = torch.rand(num_rows, generator=gen, device=device, dtype=torch.float64)
    w = (1.0 - u).clamp_min(1e-12).pow(-1.0 / (alpha - 1.0))
    # water-filling: scale the weights so that sum(min(cap, s*w)) == E
    lo, hi = 0.0, float(cap) / float(w.min())
    for _ in range(200):
        mid = 0.5 * (lo + hi)
        if float(torch.clamp(w * mid, max=cap).sum()) < num_edges:
            lo = mid
        else:
            hi = mid
    real = torch.clamp(w * hi, max=cap)
    deg = torch.floor(real).to(torch.int64)
    rem = num_edges - int(deg.sum())
    if rem > 0:  # largest fractional parts get +1 (rows below the cap)
        frac = (real - deg).masked_fill(deg >= cap, -1.0)
        deg[torch.topk(frac, rem).indices] += 1
    elif rem < 0:
        frac = (real - deg).masked_fill(deg <= 0, 2.0)
        deg[torch.topk(frac, -rem, largest=False).indices] -= 1
    if int(deg.sum()) != num_edges:
        raise RuntimeError("could not hit the requested edge count")
    return deg


_M64 = (1 << 64) - 1


def _i64(c: int) -> int:
    """A 64-bit constant as the int64 torch stores (two's complement)."""
    c &= _M64
    return c - (1 << 64) if c >= 1 << 63 else c


def _mix64(x: torch.Tensor) -> torch.Tensor:
    """splitmix64's finalizer on int64 tensors (wrapping multiplies, logical shifts):
    a counter-based hash, so edge e's column or value depends on (seed, e) only."""
    x = x ^ ((x >> 30) & ((1 << 34) - 1))
    x = x * _i64(0xBF58476D1CE4E5B9)
    x = x ^ ((x >> 27) & ((1 << 37) - 1))
    x = x * _i64(0x94D049BB133111EB)
    return x ^ ((x >> 31) & ((1 << 33) - 1))


def _key(seed: int, stream: int) -> int:
    return _i64((seed * 0x9E3779B97F4A7C15 + stream * 0xD1B54A32D192ED03) & _M64)


def synthetic_indptr(num_rows: int, num_edges: int, seed: int = 123, device="cuda",
                     alpha: float = 2.2) -> torch.Tensor:
    """indptr int32[V+1] of the synthetic graph: power-law out-degrees summing
    to num_edges (cheap: V numbers; every rank of a partitioned run computes the
    same one)."""
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    deg = powerlaw_degrees(num_rows, num_edges, gen, device, alpha)
    indptr64 = torch.zeros(num_rows + 1, dtype=torch.int64, device=device)
    indptr64[1:] = torch.cumsum(deg, 0)
    return indptr64.to(torch.int32)


def synthetic_columns(indptr: torch.Tensor, seed: int = 123, rows: tuple[int, int] | None = None,
                      self_loops: bool = False) -> torch.Tensor:
    """Columns int32 of rows [r0, r1) (all rows by default) of the synthetic
    graph with this indptr: uniform in [0, V), distinct and ascending within a
    row.  Edge e's column is a hash of (seed, e, attempt) -- duplicates within a
    row are redrawn with the next attempt at their sorted position -- so a row
    range is generated without the rest of the graph and equals the same rows
    of the whole graph (a rank of the 1-D partition builds only its block)."""
    V = indptr.numel() - 1
    r0, r1 = rows if rows is not None else (0, V)
    dev = indptr.device
    ip = indptr[r0:r1 + 1].to(torch.int64)
    e0, n = int(ip[0]), int(ip[-1] - ip[0])
    deg = ip[1:] - ip[:-1]
    row = torch.repeat_interleave(torch.arange(r0, r1, device=dev), deg, output_size=n)
    pos = torch.arange(e0, e0 + n, device=dev, dtype=torch.int64)   # global edge ids
    cols = (_mix64(pos ^ _key(seed, 0)) & ((1 << 62) - 1)) % V
    if self_loops:
        # the first slot of every non-empty row is the diagonal
        nz = deg > 0
        cols[(ip[:-1] - e0)[nz]] = torch.arange(r0, r1, device=dev)[nz]
    for attempt in range(1, 33):
        key, perm = torch.sort(row * V + cols)      # rows ascending already: stays row-major
        cols = cols[perm]
        dup = torch.zeros_like(key, dtype=torch.bool)
        dup[1:] = key[1:] == key[:-1]
        if not bool(dup.any()):
            break
        cols[dup] = (_mix64(pos[dup] ^ _key(seed, attempt)) & ((1 << 62) - 1)) % V
    else:
        raise RuntimeError("duplicate removal did not converge")
    return cols.to(torch.int32)


def synthetic_values(seed: int, e0: int, e1: int, device="cuda") -> torch.Tensor:
    """fp32 U(0,1) edge values of global edges [e0, e1) (main.cu:83-84's
    distribution), a hash of (seed, e): any slice equals the same slice of the
    whole array."""
    pos = torch.arange(e0, e1, device=device, dtype=torch.int64)
    bits = (_mix64(pos ^ _key(seed, 101)) >> 40) & ((1 << 24) - 1)   # 24 random bits
    return bits.to(torch.float32) * (1.0 / (1 << 24))


def synthetic_features(seed: int, r0: int, r1: int, dim: int, device="cuda") -> torch.Tensor:
    """fp32 U(0,1) node features (or gradient rows) of rows [r0, r1), dim wide:
    entry (r, c) is a hash of (seed, r * dim + c), so a rank of the row partition
    generates exactly its rows of the whole matrix."""
    pos = torch.arange(r0 * dim, r1 * dim, device=device, dtype=torch.int64)
    bits = (_mix64(pos ^ _key(seed, 202)) >> 40) & ((1 << 24) - 1)
    return (bits.to(torch.float32) * (1.0 / (1 << 24))).view(r1 - r0, dim)


def synthetic_csr_gpu(num_rows: int, num_edges: int, seed: int = 123, device="cuda",
                      alpha: float = 2.2, self_loops: bool = False):
    """(indptr int32[V+1], indices int32[E]) on `device`; columns uniform in
    [0, V), no duplicates within a row, ascending within a row."""
    indptr = synthetic_indptr(num_rows, num_edges, seed, device, alpha)
    return indptr, synthetic_columns(indptr, seed, self_loops=self_loops)


def small_csr(num_rows: int = 3000, seed: int = 123, extra_degrees=(0, 1, 63, 64, 65, 129, 257,
                                                                       700, 3000)):
    """Small numpy CSR with a controlled degree mix (tests)."""
    rng = np.random.default_rng(seed)
    deg = rng.integers(0, 24, size=num_rows)
    deg[rng.random(num_rows) < 0.15] = 0
    pos = rng.choice(num_rows, size=len(extra_degrees), replace=False)
    for p, d in zip(pos, extra_degrees):
        deg[p] = min(d, num_rows)
    deg[-1] = 0          # trailing empty row
    deg[0] = max(deg[0], 1)
    indptr = np.zeros(num_rows + 1, dtype=np.int64)
    indptr[1:] = np.cumsum(deg)
    indices = np.empty(indptr[-1], dtype=np.int32)
    for r in range(num_rows):
        if deg[r]:
            indices[indptr[r]:indptr[r + 1]] = np.sort(rng.choice(num_rows, size=deg[r],
                                                                  replace=False))
    return indptr.astype(np.int32), indices


def random_cbsr(num_rows: int, dim_k: int, dim_origin: int = 256, seed: int = 7):
    """Distinct selectors per row (like main.cu's std::sample) and U(0,1) data."""
    rng = np.random.default_rng(seed)
    sel = np.argsort(rng.random((num_rows, dim_origin)), axis=1)[:, :dim_k].astype(np.uint8)
    data = rng.random((num_rows, dim_k), dtype=np.float32)
    return data, sel
