"""The collective helpers of spgemm_new_amd/distributed.py on the real RCCL
("nccl") backend.

Every multi-rank test runs on gloo (CPU, or device tensors staged through host
memory by `a2a` / `ag`) or on tools/wire_model.ThreadFabric, so the branch that
hands device tensors straight to RCCL -- the one the driver's N > 1 bench takes
-- is otherwise first executed on the 8-GPU node.  RCCL refuses two ranks on
one GPU, so this runs a world-1 RCCL communicator on the one card (a
subprocess: the process group stays out of the test process) and drives the
helpers with the argument shapes the partitioned step passes: row slices at a
non-zero storage offset (one exchange round of a round-major buffer), explicit
split lists, empty rounds, uint8 CBSR records, int32 and fp32 rows,
synchronous and async_op calls (wait() then reading on the current stream),
all_gather_into_tensor, and the float64 MAX all-reduce of the collective
decisions.  Each result is compared bitwise with the copy a world-1 exchange is.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_SCRIPT = r"""
import os, sys
sys.path.insert(0, sys.argv[1])
import torch
import torch.distributed as dist
from spgemm_new_amd import distributed as D

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
assert dist.get_backend() == "nccl", dist.get_backend()
gen = torch.Generator(device=dev)
gen.manual_seed(7)
checks = 0

def same(a, b, what):
    global checks
    assert a.dtype == b.dtype and a.shape == b.shape, (what, a.shape, b.shape)
    assert torch.equal(a, b), what
    checks += 1

# a round-major exchange buffer cut into rounds: row slices at non-zero offsets
for dtype, width in ((torch.float32, 256), (torch.uint8, 160), (torch.int32, 32)):
    rows = 1000
    if dtype.is_floating_point:
        send = torch.rand((rows, width), generator=gen, device=dev)
    else:
        send = torch.randint(0, 100, (rows, width), generator=gen, device=dev).to(dtype)
    recv = torch.full((rows, width), 0, dtype=dtype, device=dev)
    cuts = [0, 0, 337, 337, 1000]            # rounds with no rows included
    works = []
    for r in range(len(cuts) - 1):
        a, b = cuts[r], cuts[r + 1]
        works.append(D.a2a(recv[a:b], send[a:b], [b - a], [b - a], async_op=True))
    for w in works:
        w.wait()
    same(recv, send, f"a2a async rounds {dtype}")
    recv.zero_()
    out = D.a2a(recv[337:], send[337:], [663], [663])
    same(out, send[337:], f"a2a sync slice {dtype}")
    same(recv[:337], torch.zeros_like(recv[:337]), f"a2a sync slice untouched {dtype}")
    out = D.a2a(recv, send)                  # no split lists
    same(out, send, f"a2a even {dtype}")

# async: the handle's wait() orders later work on the current stream after it
send = torch.rand((1 << 20, 64), generator=gen, device=dev)
recv = torch.empty_like(send)
for _ in range(3):
    ref = send.sum(dtype=torch.float64)
    w = D.a2a(recv, send, [send.shape[0]], [send.shape[0]], async_op=True)
    w.wait()
    s = recv.sum(dtype=torch.float64)        # on the current stream, after wait()
    send.add_(1.0)                           # the next round's producer
    torch.cuda.synchronize()
    assert float(s) == float(ref), (float(s), float(ref))
    checks += 1

# all_gather_into_tensor of the CBSR records (world 1: one chunk)
rec = torch.randint(0, 255, (4099, 160), generator=gen, device=dev).to(torch.uint8)
full = torch.empty_like(rec)
w = D.ag(full, rec, async_op=True)
w.wait()
same(full, rec, "ag async")
full.zero_()
same(D.ag(full, rec), rec, "ag sync")

# the MAX all-reduce of the collective decisions (float64 on the device)
t = torch.tensor([3.0, 1e12, -2.0], dtype=torch.float64, device=dev)
dist.all_reduce(t, op=dist.ReduceOp.MAX)
assert t.cpu().tolist() == [3.0, 1e12, -2.0]
checks += 1

dist.barrier()
torch.cuda.synchronize()
dist.destroy_process_group()
print(f"rccl api ok: {checks} checks")
"""


@pytest.mark.gpu
def test_collective_helpers_on_rccl(tmp_path):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29600 + os.getpid() % 300),
               RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, "-c", _SCRIPT, ROOT], capture_output=True, text=True,
                       timeout=180, env=env, cwd=str(tmp_path))
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-4000:])
    assert "rccl api ok: 18 checks" in p.stdout, p.stdout[-2000:]
