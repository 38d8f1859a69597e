import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
import bench
from langsplat_amd.graph import GraphedStep
from langsplat_amd.synthetic import CONFIGS, make_cameras, make_gaussians
c = CONFIGS["C3"]; P, W, H = c["P"], c["width"], c["height"]
dev = torch.device("cuda", 0)
model = bench.Model(make_gaussians(P, seed=0).to(dev), include_feature=True)
cam = make_cameras(1, W, H, device=dev)[0]
bg = torch.zeros(3, device=dev)
gen = torch.Generator().manual_seed(100)
gt = torch.nn.functional.normalize(torch.randn((3, H, W), generator=gen), dim=0).to(dev)
mask = (torch.rand((1, H, W), generator=gen) < 0.9).to(dev)
optim = bench.AmdAdam([{"params": [model._language_feature], "lr": 0.0025}], lr=0.0, eps=1e-15)
def fwd_bwd():
    loss = bench.render(cam, model, bench.Pipe, bg, bench.Opt, language_target=(gt, mask))["language_l1"]
    loss.backward(); return loss
g = GraphedStep(fwd_bwd, [model._language_feature]).capture()
for _ in range(10): g.replay()
torch.cuda.synchronize()
t = []
t0 = time.perf_counter()
for _ in range(20):
    a = time.perf_counter(); g.replay(); b = time.perf_counter(); optim.step(); c2 = time.perf_counter()
    t.append((b - a, c2 - b))
t1 = time.perf_counter(); torch.cuda.synchronize(); t2 = time.perf_counter()
print("host loop %.1f us/step, final sync wait %.1f us" % ((t1 - t0) / 20 * 1e6, (t2 - t1) * 1e6))
print("replay call us:", [round(x[0] * 1e6) for x in t])
print("adam call us:", [round(x[1] * 1e6) for x in t])
