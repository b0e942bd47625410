"""README-style speedup table (reference README.md:136):
MaxK SpGEMM forward and SSpMM backward at k = 8, 16, 32, 64 against dense
SpMM on the same graph and h = 256 -- our HIP dense SpMM (GNNAdvisor-style
baseline), a GNNAdvisor SAG restatement (MaxKGraph.spmm_sag, spmm_gnna.cu:60-140)
and rocSPARSE via torch.sparse.mm.  GPU only; prints one JSON line
per (graph, k) and a markdown table.

  python tools/speedup_table.py [--graphs reddit products] [--ks 8 16 32 64]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_csr_gpu  # noqa: E402


def ev_ms(fn, reps=5):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--graphs", nargs="+", default=["reddit", "products"])
    p.add_argument("--ks", nargs="+", type=int, default=[8, 16, 32, 64])
    p.add_argument("--h", type=int, default=256)
    p.add_argument("--no-vendor", action="store_true")
    args = p.parse_args()
    dev = torch.device("cuda:0")
    rows = []
    for name in args.graphs:
        V, E = CONFIGS[name]
        indptr, indices = synthetic_csr_gpu(V, E, device=dev)
        gen = torch.Generator(device=dev)
        gen.manual_seed(123)
        values = torch.rand(indices.numel(), generator=gen, device=dev)
        X = torch.rand((V, args.h), generator=gen, device=dev)
        G = torch.rand((V, args.h), generator=gen, device=dev)
        g = S.MaxKGraph(indptr, indices, values)
        dense_ms = ev_ms(lambda: g.spmm_dense(X))
        # GNNAdvisor's SAG restated (kernels/spmm_gnna.cu:60-140): unweighted, as the reference
        sag_ms = ev_ms(lambda: g.spmm_sag(X, weighted=False))
        vendor_ms = None
        if not args.no_vendor:
            a = torch.sparse_csr_tensor(indptr.long(), indices.long(), values, size=(V, V))
            try:
                vendor_ms = ev_ms(lambda: torch.sparse.mm(a, X), reps=2)
            except RuntimeError:
                vendor_ms = None
            del a
        for k in args.ks:
            data, sel = S.topk_cbsr(X, k)
            g.backward(G, sel)   # AUTO's choice first (measured once, or by rule, then cached):
            # when it reads edge selectors the forward writes them, as in a training step
            fwd_ms = ev_ms(lambda: g.forward(data, sel, args.h, edge_sel="auto"))
            bwd_ms = ev_ms(lambda: g.backward(G, sel))
            r = {"graph": name, "V": V, "E": E, "h": args.h, "k": k, "fwd_ms": round(fwd_ms, 3),
                 "bwd_ms": round(bwd_ms, 3), "bwd_algo": g.last_bwd_algo,
                 "hip_dense_ms": round(dense_ms, 3),
                 "fwd_speedup_vs_hip_dense": round(dense_ms / fwd_ms, 2),
                 "bwd_speedup_vs_hip_dense": round(dense_ms / bwd_ms, 2),
                 "gnna_sag_ms": round(sag_ms, 3),
                 "fwd_speedup_vs_gnna_sag": round(sag_ms / fwd_ms, 2),
                 "bwd_speedup_vs_gnna_sag": round(sag_ms / bwd_ms, 2)}
            if vendor_ms is not None:
                r["rocsparse_ms"] = round(vendor_ms, 3)
                r["fwd_speedup_vs_rocsparse"] = round(vendor_ms / fwd_ms, 2)
            print(json.dumps(r), flush=True)
            rows.append(r)
        del g, X, G, indptr, indices, values
        torch.cuda.empty_cache()
    print("\n| graph | k | fwd ms | bwd ms | HIP dense SpMM ms | fwd × | bwd × | GNNA SAG ms | fwd × | "
          "bwd × | rocSPARSE ms | fwd × |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    for r in rows:
        print(f"| {r['graph']} | {r['k']} | {r['fwd_ms']} | {r['bwd_ms']} | {r['hip_dense_ms']} | "
              f"{r['fwd_speedup_vs_hip_dense']} | {r['bwd_speedup_vs_hip_dense']} | "
              f"{r['gnna_sag_ms']} | {r['fwd_speedup_vs_gnna_sag']} | {r['bwd_speedup_vs_gnna_sag']} | "
              f"{r.get('rocsparse_ms', '-')} | {r.get('fwd_speedup_vs_rocsparse', '-')} |")


if __name__ == "__main__":
    main()
