"""Time the HIP CBSR producer and scatter at Reddit / products shapes (development helper)."""
import sys
import torch
sys.path.insert(0, ".")
import spgemm_new_amd as S  # noqa: E402

for V in (232965, 2449029):
    x = torch.rand((V, 256), device="cuda")
    for k in (8, 32, 64):
        for order in ("column", "value"):
            S.topk_cbsr(x, k, order=order)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(5):
                S.topk_cbsr(x, k, order=order)
            b.record()
            b.synchronize()
            ms = a.elapsed_time(b) / 5
            print(f"V={V} k={k} {order}: {ms:.3f} ms  {V * 256 * 4 / ms / 1e6:.0f} GB/s read", flush=True)

for V in (232965, 2449029):
    for k in (32,):
        x = torch.rand((V, 256), device="cuda")
        _, sel = S.topk_cbsr(x, k)
        vals = torch.rand((V, k), device="cuda")
        out = torch.empty((V, 256), device="cuda")
        S.cbsr_scatter(vals, sel, 256, out=out)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(5):
            S.cbsr_scatter(vals, sel, 256, out=out)
        b.record()
        b.synchronize()
        ms = a.elapsed_time(b) / 5
        print(f"scatter V={V} k={k}: {ms:.3f} ms  {V * 256 * 4 / ms / 1e6:.0f} GB/s written", flush=True)
