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
# the reductions above went through the direct communicator (langsplat_amd.rccl: RCCL on the caller's
# stream), unless LSR_DIRECT_RCCL=0; the deferred tail's partials + skip word: one collective
from langsplat_amd import rccl
assert (rccl._default is not None) == (os.environ.get("LSR_DIRECT_RCCL", "1") != "0"), rccl._failed
part = torch.randn((3 * P + 1,), generator=g).to(dev)
part[-1:].view(torch.int32)[0] = 0x3F800000
ref = part.clone()
direct.all_reduce_partials(part, average=True)
torch.cuda.synchronize()
assert torch.equal(part, ref)
torch.cuda.synchronize()
rccl.destroy_default()
dist.destroy_process_group()
print("RCCL_OK")
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run_child(script, timeout=110):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0", PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run([sys.executable, "-c", script], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=timeout)
    assert r.returncode == 0 and "RCCL_OK" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])


@pytest.mark.parametrize("direct", ["1", "0"])
def test_rccl_bucket_with_densification_statistics(direct, monkeypatch):
    """direct: the step's collectives through langsplat_amd.rccl (RCCL on the caller's stream) or,
    LSR_DIRECT_RCCL=0, through torch.distributed."""
    monkeypatch.setenv("LSR_DIRECT_RCCL", direct)
    _run_child(CHILD)


CAPTURED = r"""
import torch, torch.distributed as dist
from langsplat_amd.distributed import GradBucket, collective_capturable
from langsplat_amd.graph import ViewSlot
from langsplat_amd.optim import Adam
from langsplat_amd.pipeline import PipelinedGraphStep
from langsplat_amd import _native
from langsplat_amd.render import render
from langsplat_amd.synthetic import make_gaussians
from tests.test_gpu_captured_forms import _frozen_model, _overflow_views, _slot_forward, _adam, _eager_sequence
from tests.test_gpu_captured_forms import assert_states_close, _state
dist.init_process_group("nccl", rank=0, world_size=1)
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
assert collective_capturable()
# (1) the bucket's collective with the overflow flag, captured into a HIP graph and replayed
P = 5000
lang = torch.nn.Parameter(torch.zeros((P, 3), device=dev))
b = GradBucket([lang])
flag = torch.zeros((), dtype=torch.int32, device=dev)
lang.grad = torch.zeros((P, 3), device=dev)
b.all_reduce(average=True, flag=flag)  # the communicator exists before the capture
src = torch.zeros((P, 3), device=dev)
out = torch.zeros((P, 3), device=dev)
fout = torch.zeros((), device=dev)
g = torch.cuda.CUDAGraph()
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side), torch.cuda.graph(g, capture_error_mode="thread_local"):
    lang.grad.copy_(src)
    b.all_reduce(average=True, flag=flag)
    out.copy_(lang.grad)
    fout.copy_(flag.view(torch.float32))
torch.cuda.current_stream().wait_stream(side)
for k, f in enumerate((0, 0x3F800000, 0)):
    src.copy_(torch.randn((P, 3), generator=torch.Generator().manual_seed(k)).to(dev))
    flag.fill_(f)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, src), k
    assert float(fout.item()) == (1.0 if f else 0.0), (k, float(fout.item()))
# (2) PipelinedGraphStep with the bucket: one stream-A graph per step with the collective inside;
# the view over capacity skips Adam on every rank; the run equals the eager loop without that view
P = 20000
g0 = make_gaussians(P, seed=5, scale_range=(0.005, 0.04))
views = _overflow_views()
bad = 2
losses_e, se, _ = _eager_sequence(g0, [v for i, v in enumerate(views) if i != bad])
m = _frozen_model(g0)
opt = _adam(m)
R = E = 0
for i, (cam, gt, mask) in enumerate(views):
    if i == bad:
        continue
    with torch.no_grad():
        render(cam, _frozen_model(g0), type("P", (), dict(convert_SHs_python=False, compute_cov3D_python=False,
               debug=False)), torch.zeros(3, device=dev), type("O", (), dict(include_feature=True)),
               language_target=(gt, mask))
    r, e = _native.LAST_COUNTS[(P, 320, 240)]
    R, E = max(R, r), max(E, e)
S = 3
bucket = GradBucket([m._language_feature])
pg = PipelinedGraphStep(_slot_forward(m), [m._language_feature], opt, slots=[ViewSlot(*views[0]) for _ in range(S)],
                        headroom=1.0, bucket=bucket)
pg.capture(R, E, views=views[:S - 1])
assert pg.coll_in_graph and not pg.fused and all(a is None for a in pg.g_adam)
losses = []
for k in range(len(views)):
    nxt = views[k + S - 1] if k + S - 1 < len(views) else None
    losses.append(pg.replay(next_view=nxt).clone())
pg.synchronize()
torch.cuda.synchronize()
assert opt.skipped_steps() == 1
assert not pg.check() and pg.captures == 2
pg.sync()
assert int(opt.state[m._language_feature]["step"].item()) == len(views) - 1
got = [l for i, l in enumerate(losses) if i != bad]
torch.testing.assert_close(torch.stack(got), torch.stack(losses_e), rtol=1e-5, atol=0)
assert_states_close(_state(m, opt), se, "1-rank RCCL pipelined graph")
dist.destroy_process_group()
print("RCCL_OK")
"""


def test_rccl_collective_captured_in_the_step_graph():
    """VERDICT r04 item 6 / 2a on one rank: GradBucket.all_reduce(flag=) captured into a HIP graph
    (RCCL), and PipelinedGraphStep at N > 1 as one stream-A graph per step with the collective
    inside; an over-capacity view makes the step skip (the flag travels in the collective) and the
    replays equal the eager loop without that view."""
    _run_child(CAPTURED, timeout=200)
