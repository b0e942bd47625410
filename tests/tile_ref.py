"""Reference builder of the TILE plan in torch sorts (test infrastructure).

This is the plan builder spgemm_new_amd used before the device builder
(maxk_tile_plan_build, csrc/maxk_plan.hip) existed; tests/test_tile_plan.py
checks that the device builder produces the same streams bit for bit.
"""
from __future__ import annotations

import torch

from spgemm_new_amd.tile import WAVES, part_planes, ring_format


def max_group(k: int) -> int:
    return (128 if k == 32 else 64) * WAVES


def choose_shape(num_rows: int, num_cols: int, cus: int = 256,
                 k: int = 32) -> tuple[int, int, int]:
    """(num_groups, group_size, num_workgroups): groups of <= 2048 destinations
    and S <= num_rows equal source ranges each (num_workgroups = groups * S) so
    that about one workgroup runs per CU."""
    groups = -(-num_cols // max_group(k))
    splits = max(1, min(8, cus // groups, num_rows))
    # as many groups as the CUs left over allow: smaller groups, same sweep
    groups = max(groups, min(cus // splits, num_cols))
    if groups > cus:   # whole rounds of one-range workgroups
        groups = min(-(-groups // cus) * cus, num_cols)
    size = -(-num_cols // groups)
    groups = -(-num_cols // size)
    return groups, size, groups * splits


def build(indptr: torch.Tensor, indices: torch.Tensor, values: torch.Tensor, num_rows: int,
          num_cols: int, cus: int = 256, shape: tuple[int, int, int] | None = None, k: int = 32,
          record_words: int | None = None):
    """The TILE plan as a dict, or None when a chunk would overflow a wave's
    64-slot segment (many edges of few source rows into one wave's
    destinations; the other algorithms serve such graphs).  record_words: the
    record format (tile_format.h: 2 or 4; default the compiled library's)."""
    if record_words is None:
        from spgemm_new_amd.tile import record_words as _rw
        record_words = _rw()
    NB, BUF_ROWS, CHUNK_ROWS = ring_format()
    lead = NB - 1
    dev = indices.device
    E = indices.numel()
    if E == 0 or num_rows < 1 or num_cols < 1:
        return None
    if k not in (32, 64):
        return None
    G, GS, P = shape or choose_shape(num_rows, num_cols, cus, k)
    if GS > max_group(k):
        return None
    NWG = G + P - 1          # pieces (spgemm_new_amd/tile.py)
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
    wg = grp + (grp * V + rows) * P // (G * V)
    del d, j, q, grp
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
    RW = record_words
    recs = torch.zeros(total, RW, dtype=torch.int32, device=dev)

    def put(at, slot_, ring_row, vals):                                   # tile_put_record
        if RW == 2:
            w0 = slot_ | (ring_row << 24)
            recs[at, 0] = torch.where(w0 >= (1 << 31), w0 - (1 << 32), w0).to(torch.int32)
        else:
            ctl = (slot_ >> 2) | (0x0c << 8) | ((4 + (slot_ & 3)) << 16) | (0x0c << 24)
            recs[at, 0] = torch.where(ctl >= (1 << 31), ctl - (1 << 32), ctl).to(torch.int32)
            recs[at, 1] = slot_.to(torch.int32)
            recs[at, 2] = (ring_row << 10).to(torch.int32)
        recs[at, RW - 1] = vals
    every = torch.arange(total, **i64)
    put(every, torch.zeros_like(every), torch.full_like(every, BUF_ROWS - 1),
        torch.zeros(total, dtype=torch.int32, device=dev))                # padding: slot 0, zero row
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
    put(pos, so, ((c % NB) * BUF_ROWS + rin)[order], values[order].contiguous().view(torch.int32))
    del order, pos, so, seg, slot, rin, c
    # header stream: e(0) .. e(lead - 1), then e(c + lead) per chunk
    wv = torch.arange(WAVES, **i64)

    def piece_rows(cc: torch.Tensor) -> torch.Tensor:                   # cc [M] -> [NWG,16,M,3]
        li = wv[None, :, None, None] * 3 + torch.arange(3, **i64)[None, None, None, :]
        r = cc[None, None, :, None] * CHUNK_ROWS + li                     # row-list index
        ok = (li < CHUNK_ROWS) & (r < nrows[:, None, None, None])
        idx = torch.clamp(wg_start[:-1, None, None, None] + r, max=max(urow.numel() - 1, 0))
        return torch.where(ok, urow[idx].long(), -1)

    hlen = (nch + lead).repeat_interleave(WAVES)                          # [NWG*16]
    hstart = torch.cumsum(hlen, 0) - hlen
    hdrs = torch.zeros(int(hlen.sum()) + 8, 4, dtype=torch.int32, device=dev)
    # e(i) for i in [0, maxch + lead): counts of chunk i - lead, rows of chunk i
    idx_e = torch.arange(maxch + lead, **i64)
    rows_e = piece_rows(idx_e)                                            # [NWG,16,maxch+2,3]
    cnt_e = torch.zeros(NWG, WAVES, maxch + lead, **i64)
    cnt_e[..., lead:] = pad[..., 0] | (pad[..., 1] << 16)
    ok_e = idx_e[None, :] < (nch + lead)[:, None]                         # [NWG, maxch+lead]
    okw = ok_e[:, None, :].expand(NWG, WAVES, maxch + lead)
    hp = (hstart.view(NWG, WAVES, 1) + idx_e[None, None, :])[okw]
    hdrs[hp, 0] = cnt_e[okw].to(torch.int32)
    r3 = rows_e[okw]
    hdrs[hp, 1] = r3[:, 0].to(torch.int32)
    hdrs[hp, 2] = r3[:, 1].to(torch.int32)
    hdrs[hp, 3] = r3[:, 2].to(torch.int32)
    return {"headers": hdrs, "header_start": hstart.contiguous(), "records": recs,
            "record_start": rstart.contiguous(), "num_chunks": nch.to(torch.int32).contiguous(),
            "num_groups": G, "group_size": GS, "num_workgroups": P, "num_rows": V,
            "num_cols": num_cols, "k": k, "part_planes": part_planes(V, G, P),
            "zero_row": torch.zeros(256, dtype=torch.float32, device=dev)}
