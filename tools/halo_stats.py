"""Per-rank halo sizes of the 1-D row partition, computed on the
CPU the way each rank builds its block (synthetic_columns by row range) --
no collectives needed.  Bytes per step: forward records 5k B per halo node,
reverse partial sums 4k B per halo node.

    python tools/halo_stats.py [graph ...]
"""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__file__)))
from spgemm_new_amd.distributed import row_partition  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_columns, synthetic_indptr  # noqa: E402

k = 32
for graph in sys.argv[1:] or ["reddit", "products"]:
    V, E = CONFIGS[graph]
    ip = synthetic_indptr(V, E, device="cpu")
    for world in (2, 4, 8):
        b = row_partition(ip, world)
        halos = []
        for r in range(world):
            cols = synthetic_columns(ip, rows=(b[r], b[r + 1])).long()
            own = (cols >= b[r]) & (cols < b[r + 1])
            halos.append(int(torch.unique(cols[~own]).numel()))
        h = max(halos)
        print(f"{graph} N={world}: own rows/rank {V // world}, halo nodes max {h} "
              f"({h / V:.0%} of V), fwd {h * 5 * k / 1e6:.0f} MB + bwd {h * 4 * k / 1e6:.0f} MB "
              f"per rank at k={k}", flush=True)
