"""Plan of the TILE backward (maxk_sspmm_backward_tile, csrc/maxk_spgemm.hip).

The TILE backward reads every gradient row once per CU (LDS-DMA into a ring of
47-row chunks) instead of gathering k scattered floats of it per edge, and
keeps the dXs of up to 2048 destinations per workgroup in registers.  This
module builds, once per graph, the streams the kernel walks:

* destinations are cut into ``num_groups`` groups of ``group_size`` <= 2048
  columns; in a group, destination j belongs to wave ``j % 16``, slot
  ``(j // 16) >> 1`` and lane half ``(j // 16) & 1``;
* source rows are cut into ``splits`` equal ranges; workgroup
  ``b = group * splits + range``;
* a workgroup's distinct source rows (those with an edge into its group, in
  ascending order) are cut into chunks of 47 rows; chunk c sits in LDS buffer
  ``c % 3``, row 47 of every buffer is a zero row;
* per (workgroup, wave) a header stream of int32x4 entries: e(0), e(1) =
  {0, rows of chunks 0 and 1}, then e(c + 2) = {n0 | n1 << 16 of chunk c, rows
  of chunk c + 2}, where "rows" are the source rows of the wave's three DMA
  pieces (rows 3w .. 3w+2 of the chunk; -1 = the zero row);
* and a record stream: per chunk n0 records of half-0 destinations, then n1 of
  half-1 ones (each count a multiple of 4; padding record = slot 0, value 0,
  the zero row); record = int32x2 {slot | ((c % 3) * 48 + row in chunk) << 24,
  value bits}: the slot register index reads bits 7:0, the selector word is
  w >> 2, its byte offset (w << 3) & 24 and the LDS byte address of the row
  w >> 14.

The plan is built with torch sorts on the graph's device (no host loop);
``emulate`` replays it on the CPU (test infrastructure: it checks the format
against the oracle without a GPU).
"""
from __future__ import annotations

import torch

WAVES = 16
CHUNK_ROWS = 47
BUF_ROWS = 48
MAX_GROUP = 128 * WAVES     # k = 32: two destinations per slot register


def max_group(k: int) -> int:
    return (128 if k == 32 else 64) * WAVES


def choose_shape(num_cols: int, cus: int = 256, k: int = 32) -> tuple[int, int, int]:
    """(num_groups, group_size, splits): groups of <= 2048 destinations, and
    source ranges so that num_groups * splits fills about one workgroup per CU."""
    groups = -(-num_cols // max_group(k))
    splits = max(1, min(8, cus // groups))
    # as many groups as the CUs left over allow: smaller groups, same sweep
    groups = max(groups, min(cus // splits, num_cols))
    size = -(-num_cols // groups)
    groups = -(-num_cols // size)
    return groups, size, splits


def build(indptr: torch.Tensor, indices: torch.Tensor, values: torch.Tensor, num_rows: int,
          num_cols: int, cus: int = 256, shape: tuple[int, int, int] | None = None, k: int = 32):
    """The TILE plan as a dict, or None when a chunk would overflow a wave's
    64-slot segment (many edges of few source rows into one wave's
    destinations; the other algorithms serve such graphs)."""
    dev = indices.device
    E = indices.numel()
    if E == 0 or num_rows < 1 or num_cols < 1:
        return None
    if k not in (32, 64):
        return None
    G, GS, NS = shape or choose_shape(num_cols, cus, k)
    if GS > max_group(k):
        return None
    NWG = G * NS
    V = num_rows
    i64 = dict(dtype=torch.int64, device=dev)
    deg = (indptr[1:] - indptr[:-1]).long()
    rows = torch.repeat_interleave(torch.arange(V, **i64), deg)
    d = indices.long()
    grp = d // GS
    j = d - grp * GS
    w = j % WAVES
    q = j // WAVES
    if k == 32:
        slot, half = q >> 1, q & 1
    else:                                  # k = 64: one destination per slot register
        slot, half = q, torch.zeros_like(q)
    bounds = (torch.arange(NS + 1, **i64) * V) // NS
    split = torch.bucketize(rows, bounds[1:NS], right=True)
    wg = grp * NS + split
    del d, j, q, grp, split
    # distinct source rows per workgroup, and each edge's row index in that list
    key = wg * V + rows
    ukey, inv = torch.unique(key, sorted=True, return_inverse=True)
    del key
    uwg = ukey // V
    urow = (ukey - uwg * V).to(torch.int32)
    wg_start = torch.searchsorted(uwg, torch.arange(NWG + 1, **i64))
    nrows = wg_start[1:] - wg_start[:-1]
    ri = inv - wg_start[wg]
    del inv
    c = ri // CHUNK_ROWS
    rin = ri - c * CHUNK_ROWS
    del ri
    nch = (nrows + CHUNK_ROWS - 1) // CHUNK_ROWS
    maxch = max(1, int(nch.max()))
    # segments (workgroup, wave, chunk, half): record counts, padded to 4
    seg = ((wg * WAVES + w) * maxch + c) * 2 + half
    cnt = torch.bincount(seg, minlength=NWG * WAVES * maxch * 2).view(NWG, WAVES, maxch, 2)
    pad = (cnt + 3) // 4 * 4
    if int(pad.max()) > 0xFFFF:
        return None
    chunk_ok = torch.arange(maxch, **i64)[None, :] < nch[:, None]          # [NWG, maxch]
    # record stream: (workgroup, wave) major, then chunk, then half
    nrec = pad.sum(-1)                                                    # [NWG, 16, maxch]
    rlen = nrec.sum(-1).flatten()                                         # [NWG*16]
    rstart = torch.cumsum(rlen, 0) - rlen
    seg_off = rstart.view(NWG, WAVES, 1) + torch.cumsum(nrec, -1) - nrec  # first record of (wg,w,c)
    total = int(rlen.sum()) + 512                                          # + 4 KB over-read pad
    recs = torch.zeros(total, 2, dtype=torch.int32, device=dev)
    recs[:, 0] = (BUF_ROWS - 1) << 24                                     # padding: slot 0, zero row
    order = torch.argsort(seg, stable=True)
    sseg = seg[order]
    first = torch.searchsorted(sseg, sseg)
    rank = torch.arange(E, **i64) - first
    del first
    h = sseg & 1
    base_seg = sseg >> 1                                                  # (wg, w, c) flat
    pos = seg_off.flatten()[base_seg] + h * pad.view(-1, 2)[base_seg, 0] + rank
    del sseg, rank, base_seg, h
    so = slot[order]
    w0 = so | (((c % 3) * BUF_ROWS + rin)[order] << 24)
    recs[pos, 0] = torch.where(w0 >= (1 << 31), w0 - (1 << 32), w0).to(torch.int32)
    recs[pos, 1] = values[order].contiguous().view(torch.int32)
    del order, pos, so, seg, slot, rin, c
    # header stream: e(0), e(1), then e(c + 2) per chunk
    wv = torch.arange(WAVES, **i64)

    def piece_rows(cc: torch.Tensor) -> torch.Tensor:                   # cc [M] -> [NWG,16,M,3]
        li = wv[None, :, None, None] * 3 + torch.arange(3, **i64)[None, None, None, :]
        r = cc[None, None, :, None] * CHUNK_ROWS + li                     # row-list index
        ok = (li < CHUNK_ROWS) & (r < nrows[:, None, None, None])
        idx = torch.clamp(wg_start[:-1, None, None, None] + r, max=max(urow.numel() - 1, 0))
        return torch.where(ok, urow[idx].long(), -1)

    hlen = (nch + 2).repeat_interleave(WAVES)                             # [NWG*16]
    hstart = torch.cumsum(hlen, 0) - hlen
    hdrs = torch.zeros(int(hlen.sum()) + 8, 4, dtype=torch.int32, device=dev)
    # e(i) for i in [0, maxch + 2): counts of chunk i-2, rows of chunk i
    idx_e = torch.arange(maxch + 2, **i64)
    rows_e = piece_rows(idx_e)                                            # [NWG,16,maxch+2,3]
    cnt_e = torch.zeros(NWG, WAVES, maxch + 2, **i64)
    cnt_e[..., 2:] = pad[..., 0] | (pad[..., 1] << 16)
    ok_e = idx_e[None, :] < (nch + 2)[:, None]                            # [NWG, maxch+2]
    okw = ok_e[:, None, :].expand(NWG, WAVES, maxch + 2)
    hp = (hstart.view(NWG, WAVES, 1) + idx_e[None, None, :])[okw]
    hdrs[hp, 0] = cnt_e[okw].to(torch.int32)
    r3 = rows_e[okw]
    hdrs[hp, 1] = r3[:, 0].to(torch.int32)
    hdrs[hp, 2] = r3[:, 1].to(torch.int32)
    hdrs[hp, 3] = r3[:, 2].to(torch.int32)
    return {"headers": hdrs, "header_start": hstart.contiguous(), "records": recs,
            "record_start": rstart.contiguous(), "num_chunks": nch.to(torch.int32).contiguous(),
            "num_groups": G, "group_size": GS, "splits": NS, "num_rows": V, "num_cols": num_cols,
            "k": k,
            "zero_row": torch.zeros(256, dtype=torch.float32, device=dev)}


def emulate(plan, grad: torch.Tensor, sel: torch.Tensor) -> torch.Tensor:
    """CPU replay of bwd_tile_kernel over the plan (slow; small graphs): the
    LDS ring, the header and record streams and the record decode."""
    hdrs = plan["headers"].cpu()
    recs = plan["records"].cpu()
    hs = plan["header_start"].cpu().tolist()
    rs = plan["record_start"].cpu().tolist()
    nch = plan["num_chunks"].cpu().tolist()
    G, GS, NS, C = plan["num_groups"], plan["group_size"], plan["splits"], plan["num_cols"]
    grad = grad.cpu().float()
    sel = sel.cpu().long()
    K = plan.get("k", 32)
    out = torch.zeros(NS, C, K)
    if K == 32:
        jj = (2 * torch.arange(64)[:, None] + torch.arange(64)[None, :] // 32) * WAVES  # [slot, lane]
    else:
        jj = torch.arange(64)[:, None].expand(64, 64) * WAVES
    ent = torch.arange(64)[None, :] % K
    lds = torch.zeros(3 * BUF_ROWS * 256)
    for b in range(G * NS):
        sp, g = b % NS, b // NS
        d0 = g * GS
        nd = min(GS, C - d0)
        acc = torch.zeros(WAVES, 64, 64)
        ro = [rs[b * WAVES + wv] for wv in range(WAVES)]
        for c in range(nch[b]):
            for wv in range(WAVES):                    # DMA of chunk c (header e(c))
                e = hdrs[hs[b * WAVES + wv] + c]
                for i in range(3):
                    r = int(e[1 + i])
                    base = ((c % 3) * BUF_ROWS + wv * 3 + i) * 256
                    lds[base: base + 256] = 0.0 if r < 0 else grad[r]
            for wv in range(WAVES):
                e = hdrs[hs[b * WAVES + wv] + c + 2]
                n0, n1 = int(e[0]) & 0xFFFF, (int(e[0]) >> 16) & 0xFFFF
                j = jj + wv
                cols = torch.where(j < nd, sel[(d0 + j).clamp(max=C - 1), ent], 0)   # [slot, lane]
                for t in range(n0 + n1):
                    r = recs[ro[wv] + t]
                    w0 = int(r[0]) & 0xFFFFFFFF
                    val = r[1:2].view(torch.float32).item()
                    # the kernel's decode: slot = w0 & 63 (register index reads bits 7:0),
                    # selector word = w0 >> 2, byte offset = (w0 << 3) & 24, row = w0 >> 14
                    s, addr = w0 & 63, w0 >> 14
                    assert (w0 >> 6) & 0x3FFFF == 0
                    lanes = (slice(0, 64) if K == 64 else
                             slice(0, 32) if t < n0 else slice(32, 64))
                    acc[wv, s, lanes] += val * lds[addr // 4 + cols[s, lanes]]
                ro[wv] += n0 + n1
        for wv in range(WAVES):
            j = jj + wv
            m = j < nd
            out[sp, d0 + j[m], ent.expand(64, 64)[m]] = acc[wv][m]
    return out.sum(0)
