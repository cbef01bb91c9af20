"""TBD-loop bench with a world-size-1 RCCL process group created first (as bench.py's
N>1 ranks do before the context), to see whether RCCL's streams move the loop's
streams onto the caller's hardware queue.  Extra args go to bench.py."""
import os
import sys

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29517")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
t = torch.ones(1, device="cuda")
dist.all_reduce(t)
torch.cuda.synchronize()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

sys.argv = ["bench.py"] + sys.argv[1:]
bench.main()
dist.destroy_process_group()
