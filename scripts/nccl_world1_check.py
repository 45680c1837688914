"""One-rank RCCL sanity check on the GPU box: the high-priority process-group option,
all_gather_into_tensor into a slice (in place) and all_to_all_single with explicit splits,
as bench.py / lgcnhs.dist issue them."""
import os

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29561")
os.environ.setdefault("RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")
opts = dist.ProcessGroupNCCL.Options()
opts.is_high_priority_stream = True
dist.init_process_group("nccl", device_id=torch.device("cuda", 0), pg_options=opts)
buf = torch.zeros(10, 4, device="cuda")
mine = buf[2:6]
mine.fill_(3.0)
h = dist.all_gather_into_tensor(buf[2:6], mine, async_op=True)
h.wait()
x = torch.arange(12, dtype=torch.float64, device="cuda").view(6, 2)
y = torch.empty_like(x)
dist.all_to_all_single(y, x, [6], [6])
torch.cuda.synchronize()
assert torch.equal(x, y) and float(buf[2:6].sum()) == 48.0
dist.destroy_process_group()
print("nccl world-1 ok")
