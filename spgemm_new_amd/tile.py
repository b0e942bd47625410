"""Plan of the TILE backward (maxk_sspmm_backward_tile, csrc/maxk_spgemm.hip).

The TILE backward reads every gradient row once per CU (LDS-DMA into a ring of
47-row chunks) instead of gathering k scattered floats of it per edge, and
keeps the dXs of up to 2048 destinations per workgroup in registers.  This
module builds, once per graph, the streams the kernel walks:

* destinations are cut into ``num_groups`` groups of ``group_size`` <= 2048
  columns; in a group, destination j belongs to wave ``j % 16``, slot
  ``(j // 16) >> 1`` and lane half ``(j // 16) & 1``;
* the (group, source row) space x = g * V + r is cut into ``num_workgroups``
  (P) equal ranges, one per workgroup; a range crossing a group boundary holds
  one PIECE of each group it touches, run one after the other; the piece of
  (g, r) is g + floor(x * P / (G * V)) (ids 0 .. G + P - 2, csrc/tile_format.h);
  a group's first piece writes dXs, its later ones partial planes summed in
  afterwards (P = G * S: S equal source ranges per group);
* a piece's distinct source rows (those with an edge into its group, in
  ascending order) are cut into chunks of C = BR - 1 rows; chunk c sits in LDS
  buffer ``c % NB`` of a ring of NB buffers of BR rows, the last row of every
  buffer a zero row (NB, BR from ``ring_format()``; 3 x 48 by default);
* per (piece, wave) a header stream of int32x4 entries: e(0) .. e(L-1) =
  {0, rows of chunks 0 .. L-1}, then e(c + L) = {n0 | n1 << 16 of chunk c, rows
  of chunk c + L}, L = NB - 1, where "rows" are the source rows of the wave's
  three DMA pieces (rows 3w .. 3w+2 of the chunk; -1 = the zero row);
* and a record stream: per chunk n0 records of half-0 destinations, then n1 of
  half-1 ones (each count a multiple of 4; padding record = slot 0, value 0,
  the zero row); record = int32x2 {slot | ((c % NB) * BR + row in chunk) << 24,
  value bits}: the slot register index reads bits 7:0, the selector word is
  w >> 2, its byte offset (w << 3) & 24 and the LDS byte address of the row
  w >> 14.

The plan is built on the graph's device by the library
(maxk_tile_plan_build, csrc/maxk_plan.hip: two stable rocPRIM radix sorts, no
host loop); ``emulate`` replays a plan on the CPU (test infrastructure: it
checks the format against the oracle without a GPU).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib

WAVES = 16


def ring_format() -> tuple[int, int, int]:
    """(buffers, buffer rows, chunk rows) of the compiled library's TILE plan
    format (tile_format.h via maxk_tile_format)."""
    global _FMT
    if _FMT is None:
        L = _lib.load()
        nb, br = ctypes.c_int(0), ctypes.c_int(0)
        _lib.check(L.maxk_tile_format(ctypes.byref(nb), ctypes.byref(br)), "maxk_tile_format")
        _FMT = (nb.value, br.value, br.value - 1)
    return _FMT


_FMT = None


def record_words() -> int:
    """int32 words per record in the compiled library's format (2 or 4)."""
    return int(_lib.load().maxk_tile_record_words())


def max_group(k: int) -> int:
    return (128 if k == 32 else 64) * WAVES


def choose_shape(num_rows: int, num_cols: int, cus: int = 256,
                 k: int = 32) -> tuple[int, int, int]:
    """(num_groups, group_size, num_workgroups): groups of <= max_group(k)
    destinations and S <= num_rows equal source ranges each (num_workgroups =
    groups * S), about one workgroup per CU (maxk_tile_plan_shape)."""
    L = _lib.load()
    g, s, n = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
    _lib.check(L.maxk_tile_plan_shape(num_rows, num_cols, cus, k, ctypes.byref(g), ctypes.byref(s),
                                      ctypes.byref(n)), "maxk_tile_plan_shape")
    return g.value, s.value, n.value


def build(indptr: torch.Tensor, indices: torch.Tensor, values: torch.Tensor, num_rows: int,
          num_cols: int, cus: int = 256, shape: tuple[int, int, int] | None = None, k: int = 32):
    """The TILE plan as a dict (maxk_tile_plan_build on the graph's device), or
    None when a chunk would overflow a wave's 64-slot segment (many edges of
    few source rows into one wave's destinations; the other algorithms serve
    such graphs).  indptr[0] == 0 and indices / values hold exactly the graph's
    edges.  ``edge_record`` maps each CSR edge to its record, so a change of
    the graph's values is one maxk_tile_plan_set_values call (set_values)."""
    dev = indices.device
    E = indices.numel()
    if E == 0 or num_rows < 1 or num_cols < 1 or k not in (32, 64):
        return None
    G, GS, P = shape or choose_shape(num_rows, num_cols, cus, k)
    if GS > max_group(k):
        return None
    if P > G * num_rows:
        # empty workgroup ranges: their partial planes would never be written
        raise ValueError(f"TILE shape {G} groups x {num_rows} rows cannot feed {P} workgroups")
    L = _lib.load()
    NWG = G + P - 1          # pieces
    ws = torch.empty(max(1, L.maxk_tile_plan_workspace_bytes(E, G, P)), dtype=torch.uint8,
                     device=dev)
    st = _lib.stream_ptr(dev)
    sizes = (ctypes.c_int64 * 3)()
    args = (indptr.data_ptr(), indices.data_ptr(), values.data_ptr(), num_rows, num_cols, E, k,
            G, GS, P)
    _lib.check(L.maxk_tile_plan_build(*args, None, 0, None, None, 0, None, None, None, sizes,
                                      ws.data_ptr(), ws.numel(), st), "maxk_tile_plan_build(count)")
    if sizes[2] > 0xFFFF:
        return None
    i32 = dict(dtype=torch.int32, device=dev)
    i64 = dict(dtype=torch.int64, device=dev)
    hdrs = torch.empty(sizes[0], 4, **i32)
    recs = torch.empty(sizes[1], record_words(), **i32)
    hstart, rstart = torch.empty(NWG * WAVES, **i64), torch.empty(NWG * WAVES, **i64)
    nch = torch.empty(NWG, **i32)
    edge_record = torch.empty(E, **i32)
    _lib.check(L.maxk_tile_plan_build(*args, hdrs.data_ptr(), sizes[0], hstart.data_ptr(),
                                      recs.data_ptr(), sizes[1], rstart.data_ptr(), nch.data_ptr(),
                                      edge_record.data_ptr(), sizes, ws.data_ptr(), ws.numel(), st),
               "maxk_tile_plan_build")
    del ws
    return {"headers": hdrs, "header_start": hstart, "records": recs, "record_start": rstart,
            "num_chunks": nch, "edge_record": edge_record,
            "num_groups": G, "group_size": GS, "num_workgroups": P, "num_rows": num_rows,
            "num_cols": num_cols, "k": k, "part_planes": part_planes(num_rows, G, P),
            "zero_row": torch.zeros(256, dtype=torch.float32, device=dev)}


def part_planes(num_rows: int, num_groups: int, num_workgroups: int) -> int:
    """Partial planes the backward needs: the most pieces a group spans - 1."""
    return max(0, max(_group_planes(g, num_rows, num_groups, num_workgroups)
                      for g in range(num_groups)))


def _group_planes(g: int, V: int, G: int, P: int) -> int:
    return ((g + 1) * V - 1) * P // (G * V) - g * P // G


def pieces_of(b: int, V: int, G: int, P: int):
    """(piece id, group, plane) of workgroup b's pieces, in run order."""
    gv = G * V
    x0, x1 = -(-b * gv // P), -(-(b + 1) * gv // P)
    if x1 <= x0:
        return []
    return [(g + b, g, b - g * P // G) for g in range(x0 // V, (x1 - 1) // V + 1)]


def set_values(plan, values: torch.Tensor) -> None:
    """Rewrite the plan's record values from the graph's edge values (fp32[E])
    after they changed in place (maxk_tile_plan_set_values)."""
    L = _lib.load()
    _lib.check(L.maxk_tile_plan_set_values(plan["edge_record"].data_ptr(), values.data_ptr(),
                                           plan["edge_record"].numel(), plan["records"].data_ptr(),
                                           _lib.stream_ptr(values.device)),
               "maxk_tile_plan_set_values")


def emulate(plan, grad: torch.Tensor, sel: torch.Tensor) -> torch.Tensor:
    """CPU replay of bwd_tile_kernel over the plan (slow; small graphs): the
    LDS ring, the header and record streams and the record decode."""
    NB, BR, _ = ring_format()
    lead = NB - 1
    hdrs = plan["headers"].cpu()
    recs = plan["records"].cpu()
    hs = plan["header_start"].cpu().tolist()
    rs = plan["record_start"].cpu().tolist()
    nch = plan["num_chunks"].cpu().tolist()
    G, GS, P, C = plan["num_groups"], plan["group_size"], plan["num_workgroups"], plan["num_cols"]
    V = plan["num_rows"]
    grad = grad.cpu().float()
    sel = sel.cpu().long()
    K = plan.get("k", 32)
    # unwritten plane entries stay NaN and poison the result, as stale memory
    # would on the GPU (the kernel's `part` is not zeroed)
    out = torch.full((part_planes(V, G, P) + 1, C, K), float("nan"))
    if K == 32:
        jj = (2 * torch.arange(64)[:, None] + torch.arange(64)[None, :] // 32) * WAVES  # [slot, lane]
    else:
        jj = torch.arange(64)[:, None].expand(64, 64) * WAVES
    ent = torch.arange(64)[None, :] % K
    lds = torch.zeros(NB * BR * 256)
    for b, g, sp in (pc for w in range(P) for pc in pieces_of(w, V, G, P)):
        d0 = g * GS
        nd = min(GS, C - d0)
        acc = torch.zeros(WAVES, 64, 64)
        ro = [rs[b * WAVES + wv] for wv in range(WAVES)]
        for c in range(nch[b]):
            for wv in range(WAVES):                    # DMA of chunk c (header e(c))
                e = hdrs[hs[b * WAVES + wv] + c]
                for i in range(3):
                    r = int(e[1 + i])
                    row = min(wv * 3 + i, BR - 1)      # pieces past the buffer: the zero row
                    base = ((c % NB) * BR + row) * 256
                    lds[base: base + 256] = 0.0 if r < 0 else grad[r]
            for wv in range(WAVES):
                e = hdrs[hs[b * WAVES + wv] + c + lead]
                n0, n1 = int(e[0]) & 0xFFFF, (int(e[0]) >> 16) & 0xFFFF
                j = jj + wv
                cols = torch.where(j < nd, sel[(d0 + j).clamp(max=C - 1), ent], 0)   # [slot, lane]
                for t in range(n0 + n1):
                    r = recs[ro[wv] + t]
                    val = r[-1:].view(torch.float32).item()
                    if r.numel() == 2:
                        w0 = int(r[0]) & 0xFFFFFFFF
                        # the kernel's decode: slot = w0 & 63 (register index reads bits
                        # 7:0), selector word = w0 >> 2, byte offset = (w0 << 3) & 24,
                        # row = w0 >> 14
                        s, addr = w0 & 63, w0 >> 14
                        assert (w0 >> 6) & 0x3FFFF == 0
                    else:
                        # {v_perm control, slot, row address, value}: the selector register
                        # index (byte 0) and the byte the perm picks (byte 2 - 4) must name
                        # the slot's selector byte; bytes 1 and 3 select zeros
                        ctl = int(r[0]) & 0xFFFFFFFF
                        s, addr = int(r[1]), int(r[2])
                        assert ctl == (s >> 2) | 0x0c << 8 | (4 + (s & 3)) << 16 | 0x0c << 24
                        assert 0 <= s < 64 and addr % 1024 == 0
                    lanes = (slice(0, 64) if K == 64 else
                             slice(0, 32) if t < n0 else slice(32, 64))
                    acc[wv, s, lanes] += val * lds[addr // 4 + cols[s, lanes]]
                ro[wv] += n0 + n1
        for wv in range(WAVES):
            j = jj + wv
            m = j < nd
            out[sp, d0 + j[m], ent.expand(64, 64)[m]] = acc[wv][m]
    # tile_combine_kernel: dxs += group g's _group_planes(g) partial planes, in order
    res = out[0].clone()
    for g in range(G):
        d0, d1 = g * GS, min(C, (g + 1) * GS)
        for p in range(_group_planes(g, V, G, P)):
            res[d0:d1] += out[1 + p, d0:d1]
    return res
