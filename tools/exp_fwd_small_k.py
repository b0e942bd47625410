"""Products-shaped forward at k = 8 / 16 (packed CBSR records), timed alone
(median of 20 HIP-event calls).  MAXK_LIB selects a variant build.  Development tool."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_columns, synthetic_indptr, synthetic_values  # noqa: E402
from spgemm_new_amd.ops import topk_cbsr  # noqa: E402


def med(fn, n=20):
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * n)]
    for i in range(n):
        ev[2 * i].record()
        fn()
        ev[2 * i + 1].record()
    torch.cuda.synchronize()
    t = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(n))
    return t[n // 2]


dev = torch.device("cuda", 0)
GRAPH = os.environ.get("GRAPH", "products")
V, E = CONFIGS[GRAPH]
indptr = synthetic_indptr(V, E, seed=123, device=dev)
g = S.MaxKGraph(indptr, synthetic_columns(indptr, seed=123), synthetic_values(123, 0, E, device=dev))
gen = torch.Generator(device=dev)
gen.manual_seed(124)
X = torch.rand((V, 256), generator=gen, device=dev)
y = torch.empty((V, 256), device=dev)
ref = {}
for k in [int(a) for a in sys.argv[1:]] or [8, 16]:
    data, sel = topk_cbsr(X, k)
    ms = med(lambda: g.forward(data, sel, 256, out=y))
    bits = int(y.view(torch.int32).to(torch.int64).sum())   # equal sums <=> (almost surely) equal bits
    print(f"{GRAPH} k={k} fwd {ms:.3f} ms  checksum {float(y.double().sum()):.6e} bits {bits}",
          flush=True)
