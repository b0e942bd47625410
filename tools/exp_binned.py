"""Products-shaped backward algorithms at k = 8 / 16 / 32, each timed as
forward + backward (the edge-selector ones make the forward write E*k bytes):
STAGED, STAGED_EDGE, EDGE_GATHER, BINNED, BINNED_EDGE; BINNED checked against
STAGED.  Usage: python tools/exp_binned.py [k ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd import _lib  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_columns, synthetic_indptr, synthetic_values  # noqa: E402
from spgemm_new_amd.ops import _ESEL_ALGOS, topk_cbsr  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "variants_lib"))
import variants as VL  # noqa: E402  (BINNED lives in the ablation build)


def ms_of(fn, n=10):
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * n)]
    for i in range(n):
        ev[2 * i].record()
        fn()
        ev[2 * i + 1].record()
    torch.cuda.synchronize()
    t = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(n))
    return t[len(t) // 2]


def main():
    ks = [int(a) for a in sys.argv[1:]] or [8, 16]
    only = os.environ.get("ALGOS")          # e.g. ALGOS=binned_edge,edge_gather
    dev = torch.device("cuda", 0)
    V, E = CONFIGS["products"]
    t0 = time.time()
    indptr = synthetic_indptr(V, E, seed=123, device=dev)
    indices = synthetic_columns(indptr, seed=123)
    values = synthetic_values(123, 0, E, device=dev)
    g = S.MaxKGraph(indptr, indices, values)
    t1 = time.time()
    plan = VL.bin_plan(g)
    torch.cuda.synchronize()
    print(f"graph {time.time() - t0:.1f}s, bin plan {time.time() - t1:.2f}s: slots "
          f"{plan['num_slots']} ({plan['num_slots'] / E:.4f} per edge), bins {plan['num_bins']}",
          flush=True)
    gen = torch.Generator(device=dev)
    gen.manual_seed(124)
    X = torch.rand((V, 256), generator=gen, device=dev)
    G = torch.rand((V, 256), generator=gen, device=dev)
    y = torch.empty((V, 256), device=dev)
    names = {_lib.MAXK_BWD_STAGED: "staged", _lib.MAXK_BWD_STAGED_EDGE: "staged_edge",
             _lib.MAXK_BWD_EDGE_GATHER: "edge_gather", VL.MAXK_BWD_BINNED: "binned",
             VL.MAXK_BWD_BINNED_EDGE: "binned_edge"}
    for k in ks:
        data, sel = topk_cbsr(X, k)
        dx = torch.empty((V, k), device=dev)
        ref = g.backward(G, sel, algo=_lib.MAXK_BWD_STAGED).clone()
        for a, name in names.items():
            if a == _lib.MAXK_BWD_EDGE_GATHER and k not in (8, 16, 32):
                continue
            if only and name not in only.split(","):
                continue
            esel = a in _ESEL_ALGOS or a == VL.MAXK_BWD_BINNED_EDGE
            f = ms_of(lambda: g.forward(data, sel, 256, out=y, edge_sel=esel))
            if a in (VL.MAXK_BWD_BINNED, VL.MAXK_BWD_BINNED_EDGE):
                b = ms_of(lambda: VL.backward_binned(g, G, sel, plan,
                                                     edge=a == VL.MAXK_BWD_BINNED_EDGE, out=dx))
            else:
                b = ms_of(lambda: g.backward(G, sel, out=dx, algo=a))
            err = float(((dx - ref).abs() / ref.abs().clamp_min(1)).max())
            print(f"k={k} {name:12s} fwd {f:.3f} bwd {b:.3f} sum {f + b:.3f} ms  rel {err:.2e}",
                  flush=True)
        g._ws.clear()
        g._esel.clear()


if __name__ == "__main__":
    main()
