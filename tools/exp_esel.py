"""Products (config 3): forward with / without edge selectors, and the
backward algorithms including STAGED_EDGE, each the minimum of 5 timed calls;
the forward pair is measured three times, interleaved."""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__file__)))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd import _lib, ops  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_csr_gpu  # noqa: E402

dev = torch.device("cuda")
graph = sys.argv[1] if len(sys.argv) > 1 else "products"
V, E = CONFIGS[graph]
ip, ix = synthetic_csr_gpu(V, E, device=dev)
gen = torch.Generator(device=dev)
gen.manual_seed(1)
vals = torch.rand(E, generator=gen, device=dev)
X = torch.rand((V, 256), generator=gen, device=dev)
G = torch.rand((V, 256), generator=gen, device=dev)
g = S.MaxKGraph(ip, ix, vals)
print("lib", _lib.LIB_PATH)
for k in [int(a) for a in sys.argv[2:]] or (8, 16, 32):
    data, sel = S.topk_cbsr(X, k)
    y = torch.empty((V, 256), device=dev)
    dx = torch.empty((V, k), device=dev)
    fw = []
    for _ in range(3):
        f0 = ops._min_ms(lambda: g.forward(data, sel, 256, out=y, edge_sel=False), 5)
        f1 = ops._min_ms(lambda: g.forward(data, sel, 256, out=y, edge_sel=True), 5)
        fw.append(f"{f0:.3f}/{f1:.3f}")
    res = {}
    for name, a in (("atomic", _lib.MAXK_BWD_ATOMIC), ("staged", _lib.MAXK_BWD_STAGED),
                    ("staged_edge", _lib.MAXK_BWD_STAGED_EDGE),
                    ("edge_gather", _lib.MAXK_BWD_EDGE_GATHER)):
        res[name] = ops._min_ms(lambda: g.backward(G, sel, out=dx, algo=a), 5)
    print(f"{graph} k={k}: fwd plain/esel {' '.join(fw)} | " +
          " ".join(f"{n} {t:.3f}" for n, t in res.items()), flush=True)
