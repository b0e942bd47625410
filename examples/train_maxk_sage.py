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
    python examples/train_maxk_sage.py --graph proteins --relations 8 --steps 20

With --relations R the graph carries R edge features (ogbn-proteins has 8) and
every layer aggregates all of them with one fused SpGEMM (SpGEMMMultiFunction,
BASELINE config 5) followed by a neighbour weight per relation.

Multi-GPU (one process per GPU, RCCL): the graph is 1-D row-partitioned
(spgemm_new_amd.distributed.PartitionedMaxK), each rank trains on its own rows
with PartitionedSpGEMMFunction (halo CBSR exchange in the forward, halo partial
sums back in the backward) and the replicated Linear weights' gradients are
all-reduced:

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        examples/train_maxk_sage.py --graph reddit --steps 20
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
from spgemm_new_amd.layers import MaxKRelSAGELayer, MaxKSAGELayer  # noqa: E402


class MaxKSAGE(nn.Module):
    """Linear -> [MaxK-SAGE layer, dropout, norm] x L -> Linear (utils/models.py:199-257).
    num_rel > 1: the multi-relation layer (one fused aggregation for R edge
    features, a neighbour weight per relation)."""

    def __init__(self, in_size, hid_size, out_size, num_layers, maxk, dropout=0.5, num_rel=1):
        super().__init__()
        self.num_rel = num_rel
        self.lin_in = nn.Linear(in_size, hid_size)
        self.layers = nn.ModuleList(
            MaxKSAGELayer(hid_size, maxk) if num_rel == 1 else
            MaxKRelSAGELayer(hid_size, maxk, num_rel) for _ in range(num_layers))
        self.norms = nn.ModuleList(nn.LayerNorm(hid_size) for _ in range(num_layers))
        self.drop = nn.Dropout(dropout)
        self.lin_out = nn.Linear(hid_size, out_size)

    def forward(self, graph, x, values=None):
        """graph: the (indptr, indices, values) tuple ((indptr, indices) plus
        values fp32[E, R] with relations), or a rank's PartitionedMaxK (x then
        holds the rank's own rows)."""
        x = self.lin_in(x)
        for layer, norm in zip(self.layers, self.norms):
            h = layer(graph, x) if self.num_rel == 1 else layer(graph, x, values)
            x = norm(self.drop(h))
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
    p.add_argument("--relations", type=int, default=1,
                   help="R > 1: R edge-feature relations, fused multi-relation aggregation")
    p.add_argument("--backend", default=os.environ.get("BENCH_BACKEND", "nccl"),
                   help="torch.distributed backend when WORLD_SIZE > 1 (nccl = RCCL)")
    args = p.parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dist = None
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) %
                       max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    if world > 1:
        import torch.distributed as dist
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)
    V, E = CONFIGS[args.graph]
    if args.nodes:
        E, V = int(E * args.nodes / V), args.nodes
    indptr, indices = synthetic_csr_gpu(V, E, device=dev)
    R = args.relations
    if R == 1:
        values = torch.ones(indices.numel(), device=dev)      # sum aggregation (utils/models.py:227)
    else:                                                     # R synthetic edge features in [0, 1)
        g0 = torch.Generator(device=dev)
        g0.manual_seed(1)
        values = torch.rand((indices.numel(), R), generator=g0, device=dev) / R
    gen = torch.Generator(device=dev)
    gen.manual_seed(0)
    feats = torch.randn((V, args.feat), generator=gen, device=dev)
    w = torch.randn((args.feat, args.classes), generator=gen, device=dev)
    labels = (feats @ w).argmax(1)                              # learnable synthetic labels
    torch.manual_seed(0)                                          # same initial weights on every rank
    model = MaxKSAGE(args.feat, args.hidden, args.classes, args.layers, args.maxk,
                     num_rel=R).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=args.lr)
    graph = (indptr, indices, values) if R == 1 else (indptr, indices)
    if dist is not None:
        from spgemm_new_amd.distributed import PartitionedMaxK
        graph = PartitionedMaxK(indptr, indices, values, rank, world, dev)
        feats, labels = graph.local_rows(feats), graph.local_rows(labels)
    losses, times = [], []
    for step in range(args.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        # mean over ALL nodes: each rank sums its own rows' losses, divided by V
        out = model(graph, feats) if R == 1 or dist is not None else model(graph, feats, values)
        loss = F.cross_entropy(out, labels, reduction="sum") / V
        loss.backward()
        if dist is not None:   # replicated weights: sum the ranks' gradients
            grads = [q.grad for q in model.parameters() if q.grad is not None]
            flat = torch.cat([g.reshape(-1) for g in grads])
            dist.all_reduce(flat)
            off = 0
            for g in grads:
                g.copy_(flat[off:off + g.numel()].view_as(g))
                off += g.numel()
            loss = loss.detach().clone()
            dist.all_reduce(loss)
        opt.step()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        losses.append(float(loss))
        if rank == 0:
            print(f"step {step:3d}  loss {losses[-1]:.4f}  {times[-1] * 1e3:.1f} ms", flush=True)
    steady = times[2:] or times
    if rank == 0:
        print(f"{args.graph}: V={V} E={indices.numel()} layers={args.layers} hidden={args.hidden} "
              f"k={args.maxk} relations={R} gpus={world}: "
              f"{sum(steady) / len(steady) * 1e3:.1f} ms/step, "
              f"loss {losses[0]:.3f} -> {losses[-1]:.3f}")
    if dist is not None:
        dist.destroy_process_group()
    return losses


if __name__ == "__main__":
    main()
