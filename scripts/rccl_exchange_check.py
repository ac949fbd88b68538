"""One-GPU RCCL check of the N > 1 record exchanges (world size 1: the
collectives are copies, but they run through RCCL on device buffers and the
communication stream exactly as bench.py issues them)."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "svt-av1-mirror_amd"))
import svtme_dist as D  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
comm = torch.cuda.Stream()
local = torch.randint(0, 256, (4 * 1000,), dtype=torch.uint8, device="cuda")
out = torch.empty_like(local)
ev = torch.cuda.Event()
ev.record()
comm.wait_event(ev)
D.exchange_to_owners_device(local, out, dist, stream=comm)
g = torch.empty_like(local)
D.gather_chunks_device(local, g, dist, stream=comm)
torch.cuda.synchronize()
assert torch.equal(out, local) and torch.equal(g, local)
for q in range(4):
    assert torch.equal(D.owned_picture_records(out, 1, 4, q, 900), local[q * 1000: q * 1000 + 900])
dist.destroy_process_group()
print("rccl exchange check OK")
