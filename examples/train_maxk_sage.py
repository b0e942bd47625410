#!/usr/bin/env python3
"""MaxK-GNN SAGE training on one MI355X with the HIP aggregation path.

Mirrors the reference model's layer flow (utils/models.py SAGE.forward:
Linear -> [MaxK + SpGEMM aggregation, self + neighbour linear] x L -> Linear),
with SpGEMMFunction.apply(x, (indptr, indices, values), k) as the fused MaxK +
aggregation op -- the call the reference makes -- on a synthetic graph of a
BASELINE shape.  DGL and the datasets are not available offline, so the graph
and the node labels are synthetic (labels are a function of the features, so
the loss can fall).

    python examples/train_maxk_sage.py --graph reddit --steps 20
"""
import argparse
import os
import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spgemm_new_amd.graphs import CONFIGS, synthetic_csr_gpu  # noqa: E402
from spgemm_new_amd.models import SpGEMMFunction  # noqa: E402


class MaxKSAGE(nn.Module):
    def __init__(self, in_size, hid_size, out_size, num_layers, maxk, dropout=0.5):
        super().__init__()
        self.maxk = maxk
        self.lin_in = nn.Linear(in_size, hid_size)
        self.fc_self = nn.ModuleList(nn.Linear(hid_size, hid_size) for _ in range(num_layers))
        self.fc_neigh = nn.ModuleList(nn.Linear(hid_size, hid_size) for _ in range(num_layers))
        self.norms = nn.ModuleList(nn.LayerNorm(hid_size) for _ in range(num_layers))
        self.drop = nn.Dropout(dropout)
        self.lin_out = nn.Linear(hid_size, out_size)

    def forward(self, graph, x):
        x = self.lin_in(x)
        for fs, fn, norm in zip(self.fc_self, self.fc_neigh, self.norms):
            x_agg = SpGEMMFunction.apply(x, graph, self.maxk)   # MaxK + SpGEMM (HIP)
            x = norm(self.drop(fs(x) + fn(x_agg)))
        return self.lin_out(x)


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--graph", default="reddit", choices=sorted(CONFIGS))
    p.add_argument("--nodes", type=int, default=None, help="override V (E scaled by the degree)")
    p.add_argument("--hidden", type=int, default=256)
    p.add_argument("--maxk", type=int, default=32)
    p.add_argument("--layers", type=int, default=3)
    p.add_argument("--feat", type=int, default=602)
    p.add_argument("--classes", type=int, default=41)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--lr", type=float, default=1e-2)
    args = p.parse_args(argv)
    dev = torch.device("cuda:0")
    V, E = CONFIGS[args.graph]
    if args.nodes:
        E, V = int(E * args.nodes / V), args.nodes
    indptr, indices = synthetic_csr_gpu(V, E, device=dev)
    values = torch.ones(indices.numel(), device=dev)          # sum aggregation (utils/models.py:227)
    gen = torch.Generator(device=dev)
    gen.manual_seed(0)
    feats = torch.randn((V, args.feat), generator=gen, device=dev)
    w = torch.randn((args.feat, args.classes), generator=gen, device=dev)
    labels = (feats @ w).argmax(1)                              # learnable synthetic labels
    model = MaxKSAGE(args.feat, args.hidden, args.classes, args.layers, args.maxk).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=args.lr)
    graph = (indptr, indices, values)
    losses, times = [], []
    for step in range(args.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        loss = F.cross_entropy(model(graph, feats), labels)
        loss.backward()
        opt.step()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        losses.append(float(loss))
        print(f"step {step:3d}  loss {losses[-1]:.4f}  {times[-1] * 1e3:.1f} ms", flush=True)
    steady = times[2:] or times
    print(f"{args.graph}: V={V} E={indices.numel()} layers={args.layers} hidden={args.hidden} "
          f"k={args.maxk}: {sum(steady) / len(steady) * 1e3:.1f} ms/step, "
          f"loss {losses[0]:.3f} -> {losses[-1]:.3f}")
    return losses


if __name__ == "__main__":
    main()
