#!/usr/bin/env python3
"""Config 5 (proteins R=8, k=32, h=256): the fused forward and the multi-relation
STAGED backward in their LDS, register ("gather") and bank-ordered ("banked") forms, each run a few times
so a rocprofv3 pass can attribute counters per kernel.  Development tool.

usage: tools/exp_multi_forms.py [--reps 5]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd import _lib  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_columns, synthetic_indptr, synthetic_values  # noqa: E402
from spgemm_new_amd.ops import _min_ms  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "variants_lib"))
import variants as VL  # noqa: E402  (the ablation build: register / bank-ordered forms)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="", help="comma-separated subset of the forms' names")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    V, E = CONFIGS["proteins"]
    R, k, h = 8, 32, 256
    indptr = synthetic_indptr(V, E, seed=123, device=dev)
    indices = synthetic_columns(indptr, seed=123)
    vals = torch.stack([synthetic_values(130 + q, 0, E, device=dev) for q in range(R)],
                       dim=1).contiguous()
    g = S.MaxKGraph(indptr, indices, vals[:, 0].contiguous())
    gen = torch.Generator(device=dev)
    gen.manual_seed(124)
    X = torch.rand((V, h), generator=gen, device=dev)
    G = torch.rand((R, V, h), generator=gen, device=dev)
    data, sel = S.topk_cbsr(X, k)
    y = torch.empty((R, V, h), device=dev)
    dx = torch.empty((V, k), device=dev)
    ms, me = _lib.MAXK_BWD_MULTI_STAGED, _lib.MAXK_BWD_MULTI_EDGE_GATHER
    calls = {
        "fwd lds": lambda: g.forward_multi(data, sel, vals, h, out=y),
        "fwd gather": lambda: VL.forward_multi_gather(g, data, sel, vals, h, out=y),
        "bwd lds": lambda: g.backward_multi(G, sel, vals, out=dx, algo=ms),
        "bwd regs": lambda: VL.backward_multi_form(g, G, sel, vals, "gather", False, out=dx),
        "bwd banked": lambda: VL.backward_multi_form(g, G, sel, vals, "banked", False, out=dx),
        "bwd eg lds": lambda: g.backward_multi(G, sel, vals, out=dx, algo=me),
        "bwd eg banked": lambda: VL.backward_multi_form(g, G, sel, vals, "banked", True, out=dx),
    }
    only = [x.strip() for x in a.only.split(",") if x.strip()]
    for name, fn in calls.items():
        if only and name not in only:
            continue
        print(f"{name}: {_min_ms(fn, reps=a.reps):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
