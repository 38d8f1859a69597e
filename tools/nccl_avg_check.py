"""RCCL check on one GPU (world size 1): GradBucket.all_reduce(average=True) takes ReduceOp.AVG on
the nccl backend; this confirms the op exists in the installed RCCL and leaves the values intact.

    python tools/nccl_avg_check.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import os, torch, torch.distributed as dist
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29533")
os.environ.setdefault("RANK", "0"); os.environ.setdefault("WORLD_SIZE", "1")
torch.cuda.set_device(0)
dist.init_process_group("nccl")
from langsplat_amd.distributed import GradBucket
p = torch.nn.Parameter(torch.zeros(1000, 3, device="cuda"))
q = torch.nn.Parameter(torch.zeros(10, 1, device="cuda"))
b = GradBucket([p, q]); b.flat.fill_(2.0)  # flat bucket (several parameters)
b.all_reduce(average=True); torch.cuda.synchronize()
print("avg ok", dist.get_backend(), float(b.flat[0]), torch.equal(b.flat, torch.full_like(b.flat, 2.0)))
d = GradBucket([p]); p.grad = torch.full((1000, 3), 2.0, device="cuda")  # direct mode (one parameter)
d.all_reduce(average=True); torch.cuda.synchronize()
print("direct avg ok", torch.equal(p.grad, torch.full_like(p.grad, 2.0)))
dist.destroy_process_group()
