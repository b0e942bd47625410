"""Reference restatement of the BINNED backward's plan and of its two phases
(test infrastructure; the ablation library builds the plan on the device,
maxk_bin_plan_build in tools/variants_lib/maxk_variants_plan.hip).

Plan (tools/variants_lib/maxk_variants.h, BINNED): destination bin b = columns
[b*255, b*255 + 255); a bin's in-edges ordered by (XCD of the edge's phase-1
panel = (panel // 4) % 8, edge id), then packed first-fit into windows of 64
slots with distinct destinations, at most 8 windows open (the oldest closed,
padded, when an edge fits none); windows numbered in opening order; padding
slots hold destination 0xFF.  Plain Python loops: small graphs only.
"""
from __future__ import annotations

import numpy as np

DESTS, WINDOW, OPEN, XCDS, PANEL_WAVES = 255, 64, 8, 8, 4


def edge_panels(panel_start: np.ndarray, num_edges: int) -> np.ndarray:
    """Panel of each edge: the last panel whose first edge is <= e
    (panel_start = the schedule's edge coordinates, num_panels + 1 of them)."""
    starts = np.asarray(panel_start[:-1], dtype=np.int64)
    return np.searchsorted(starts, np.arange(num_edges), side="right") - 1


def build(panel_start: np.ndarray, indices: np.ndarray, num_cols: int):
    """(bin_pos int32[E], bin_ptr int32[nb+1], bin_dst uint8[slots], slots)."""
    indices = np.asarray(indices, dtype=np.int64)
    E = len(indices)
    nb = -(-num_cols // DESTS)
    xcd = (edge_panels(panel_start, E) // PANEL_WAVES) % XCDS
    key = (indices // DESTS) * XCDS + xcd
    order = np.argsort(key, kind="stable")
    bins = key[order] // XCDS
    starts = np.searchsorted(bins, np.arange(nb + 1), side="left")
    per_bin = []
    for b in range(nb):
        windows = 0
        placed = []            # (edge, window, fill)
        open_ = []             # [window id, fill, set of dests]
        for q in range(starts[b], starts[b + 1]):
            e = int(order[q])
            d = int(indices[e] - b * DESTS)
            i = next((j for j, w in enumerate(open_) if d not in w[2]), None)
            if i is None:
                if len(open_) == OPEN:
                    open_.pop(0)
                open_.append([windows, 0, set()])
                windows += 1
                i = len(open_) - 1
            w = open_[i]
            placed.append((e, w[0], w[1], d))
            w[1] += 1
            w[2].add(d)
            if w[1] == WINDOW:
                open_.pop(i)
        per_bin.append((windows, placed))
    ptr = np.zeros(nb + 1, dtype=np.int64)
    ptr[1:] = np.cumsum([w for w, _ in per_bin]) * WINDOW
    slots = int(ptr[-1])
    pos = np.full(E, -1, dtype=np.int64)
    dst = np.full(slots, 0xFF, dtype=np.uint8)
    for b, (_, placed) in enumerate(per_bin):
        for e, w, f, d in placed:
            s = ptr[b] + w * WINDOW + f
            pos[e] = s
            dst[s] = d
    return pos.astype(np.int32), ptr.astype(np.int32), dst, slots


def backward(indptr, indices, values, grad, sel, num_cols, plan, edge_selectors=None):
    """Both phases in fp32 as the kernels do them: P[bin_pos[e]] = val[e] *
    G[row(e), sel[c]] (selectors >= h read 0), then per bin the slots added
    in slot order into the destination rows.  Returns dXs fp32[num_cols, k]."""
    pos, ptr, dst, slots = plan
    grad = np.asarray(grad, dtype=np.float32)
    sel = np.asarray(sel)
    k = sel.shape[1]
    h = grad.shape[1]
    E = len(indices)
    rows = np.repeat(np.arange(len(indptr) - 1), np.diff(indptr))
    esel = sel[indices] if edge_selectors is None else edge_selectors.reshape(E, k)
    gpad = np.zeros((grad.shape[0], 256), dtype=np.float32)
    gpad[:, :h] = grad
    P = np.zeros((slots, k), dtype=np.float32)
    P[pos] = np.asarray(values, np.float32)[:, None] * gpad[rows[:, None], esel]
    out = np.zeros((num_cols, k), dtype=np.float32)
    for b in range(len(ptr) - 1):
        for s in range(ptr[b], ptr[b + 1]):
            if dst[s] != 0xFF:
                c = b * DESTS + int(dst[s])
                out[c] += P[s]
    return out
