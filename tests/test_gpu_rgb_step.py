"""The RGB stage's train step end to end (VERDICT r02 missing item 4; train.py:76-138 with
include_feature=False): bench.RGBStep -- render() on the fused path, (1 - 0.2) L1 + 0.2 (1 - SSIM) on
the colour image (train.py:100-103), backward through every geometry and appearance gradient, the
densification statistics kernel (train.py:125-126), one Adam launch over the six groups
(scene/gaussian_model.py:219-226) -- against the same step written as the reference writes it:
GaussianModel's torch activations into GaussianRasterizer (LANGSPLAT_AMD_FUSED=0), torch autograd,
the densification statistics as torch ops.  Gradients within the parity tolerance (the two paths'
activations differ by a few ulp), statistics equal, every parameter moved by at most its lr (Adam's
first step)."""
import numpy as np
import pytest
import torch

import bench
from langsplat_amd.render import render
from langsplat_amd.synthetic import make_cameras, make_gaussians
from tests.test_gpu_parity import assert_grad_close

pytestmark = pytest.mark.gpu
DEV = "cuda"
GROUPS = {"xyz": "_xyz", "f_dc": "_features_dc", "f_rest": "_features_rest", "opacity": "_opacity",
          "scaling": "_scaling", "rotation": "_rotation"}


def test_rgb_step_matches_reference_ops(monkeypatch):
    W, H, P = 128, 96, 3000
    params = make_gaussians(P, seed=16, scale_range=(0.02, 0.12)).to(DEV)
    cam = make_cameras(1, W, H, device=DEV)[0]
    gt = torch.rand((3, H, W), generator=torch.Generator().manual_seed(5)).to(DEV)

    # the reference's formulation
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "0")
    ref = bench.Model(make_gaussians(P, seed=16, scale_range=(0.02, 0.12)).to(DEV), include_feature=False)
    pkg = render(cam, ref, bench.Pipe, torch.zeros(3, device=DEV), bench.OptRGB)
    image = pkg["render"]
    loss_ref = (0.8 * torch.abs(image - gt).mean() + 0.2 * (1.0 - bench.ssim(image, gt)))
    loss_ref.backward()
    vis = pkg["visibility_filter"]
    vg = pkg["viewspace_points"].grad
    max_r = torch.zeros((P,), device=DEV)
    accum, denom = torch.zeros((P, 1), device=DEV), torch.zeros((P, 1), device=DEV)
    max_r[vis] = torch.max(max_r[vis], pkg["radii"][vis])
    accum[vis] += torch.norm(vg[vis, :2], dim=-1, keepdim=True)
    denom[vis] += 1

    # bench.py's step (fused path), the gradients captured as Adam receives them
    monkeypatch.setenv("LANGSPLAT_AMD_FUSED", "1")
    step = bench.RGBStep(params, cam, gt)
    before = {k: getattr(step.model, a).detach().clone() for k, a in GROUPS.items()}
    got = {}
    orig = step.optim.step

    def spy(*a, **kw):
        for grp in step.optim.param_groups:
            got[grp["name"]] = grp["params"][0].grad.detach().clone()
        return orig(*a, **kw)
    step.optim.step = spy
    loss = step()
    torch.cuda.synchronize()
    torch.testing.assert_close(loss.detach(), loss_ref.detach(), rtol=1e-5, atol=0)
    for k, a in GROUPS.items():
        assert_grad_close(k, got[k].cpu().numpy(), getattr(ref, a).grad.cpu().numpy())
        lr = next(g["lr"] for g in step.optim.param_groups if g["name"] == k)
        moved = (getattr(step.model, a).detach() - before[k]).abs()
        assert float(moved.max()) <= lr * (1 + 1e-4) and float(moved.max()) > 0, k
        assert getattr(step.model, a).grad is None  # zero_grad(set_to_none=True)
    torch.testing.assert_close(step.max_radii2D, max_r, rtol=0, atol=0)
    torch.testing.assert_close(step.denom, denom, rtol=0, atol=0)
    assert_grad_close("xyz_gradient_accum", step.xyz_gradient_accum.cpu().numpy(), accum.cpu().numpy())
    assert int(vis.sum()) > 0 and np.isfinite(float(loss.detach()))
