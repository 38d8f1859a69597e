"""The RCCL collective path on a GPU (the all-reduce was never exercised by
the GPU suite).  One rank over backend "nccl" (= RCCL on ROCm) on cuda:0, in a child process so a
communicator problem cannot take the test runner with it: GradBucket's flat bucket with the
densification statistics (RCCL ncclAvg, then the MAX of max_radii2D) and its direct mode, against
the same values computed without a collective.  With one rank the averaged bucket must come back
bit-identical, which checks that ncclAvg divides by the world size and that the statistics slots
round-trip through apply_densification exactly.  Multi-rank sums are covered with gloo on CPU
(tests/test_distributed.py); the 8-GPU node is the driver's."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os, torch, torch.distributed as dist
from langsplat_amd.distributed import GradBucket
dist.init_process_group("nccl", rank=0, world_size=1)
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
g = torch.Generator().manual_seed(3)
P = 5000
xyz = torch.nn.Parameter(torch.zeros((P, 3), device=dev))
opac = torch.nn.Parameter(torch.zeros((P, 1), device=dev))
bucket = GradBucket([xyz, opac], densify_points=P)
gx = torch.randn((P, 3), generator=g).to(dev)
go = torch.randn((P, 1), generator=g).to(dev)
xyz.grad.add_(gx)
opac.grad.add_(go)
radii = (torch.randint(-2, 9, (P,), generator=g).clamp_(min=0)).to(torch.int32).to(dev)
vgrad = torch.randn((P, 3), generator=g).to(dev)
max_r = torch.rand((P,), generator=g).mul_(4).to(dev)
max_r0 = max_r.clone()
bucket.stage_densification(radii, vgrad, max_r)
bucket.all_reduce(average=True)
torch.cuda.synchronize()
assert dist.get_backend() == "nccl"
assert bucket._divided_by == 1
assert torch.equal(xyz.grad, gx) and torch.equal(opac.grad, go), "ncclAvg over one rank changed the bucket"
vis = radii > 0
ref_r = max_r0.clone()
ref_r[vis] = torch.max(ref_r[vis], radii[vis].float())
assert torch.equal(max_r, ref_r), "max_radii2D"
acc = torch.zeros((P, 1), device=dev)
den = torch.zeros((P, 1), device=dev)
bucket.apply_densification(acc, den)
ref_acc = torch.zeros((P, 1), device=dev)
ref_acc[vis] += torch.norm(vgrad[vis, :2], dim=-1, keepdim=True)
torch.testing.assert_close(acc, ref_acc, rtol=1e-6, atol=0)
assert torch.equal(den.view(-1), vis.float()), "denom"
# direct mode (the language step): the .grad autograd hands over is reduced in place
lang = torch.nn.Parameter(torch.zeros((P, 3), device=dev))
direct = GradBucket([lang])
assert direct.direct
gl = torch.randn((P, 3), generator=g).to(dev)
lang.grad = gl.clone()
direct.all_reduce(average=True)
torch.cuda.synchronize()
assert torch.equal(lang.grad, gl)
lang.grad = None  # a rank whose parameter got no gradient joins with zeros
direct.all_reduce(average=False)
torch.cuda.synchronize()
assert lang.grad is not None and not lang.grad.any()
dist.destroy_process_group()
print("RCCL_OK")
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_rccl_bucket_with_densification_statistics():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0", PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run([sys.executable, "-c", CHILD], cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "RCCL_OK" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
