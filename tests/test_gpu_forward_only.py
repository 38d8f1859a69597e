"""The inference form (VERDICT r03 missing item 3): render.py renders under torch.no_grad()
(/root/reference/render.py:24-55), and then the rasterizer's autograd wrapper passes
LSR_FWD_NO_BACKWARD (include/lsr.h), so the compositing kernel writes the images only -- no cover
masks, split-replay states, backward work lists, final T or contributor counts.  The images, radii
and the fused loss must be bit-identical to the training forward's; a backward of such a forward is
refused under settings.debug."""
import numpy as np
import pytest
import torch

import bench
from langsplat_amd import _native
from langsplat_amd.synthetic import CONFIGS, make_cameras, make_gaussians
from tests.scenes import scene, to_device

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _spy_flags(monkeypatch):
    """Record the forward flags every native forward call receives (the NO_BACKWARD path
    must really be taken under torch.no_grad(), not only produce the same images)."""
    seen = []
    real = _native.rasterize_gaussians

    def spy(*a, **kw):
        seen.append(int(kw.get("flags", 0)))
        return real(*a, **kw)
    monkeypatch.setattr(_native, "rasterize_gaussians", spy)
    return seen


@pytest.mark.parametrize("with_loss", [False, True])
def test_inference_forward_matches_training_forward_c3(with_loss, monkeypatch):
    seen = _spy_flags(monkeypatch)
    c = CONFIGS["C3"]
    P, W, H = c["P"], c["width"], c["height"]
    model = bench.Model(make_gaussians(P, seed=0).to(DEV), include_feature=True)
    cam = make_cameras(1, W, H, device=DEV)[0]
    bg = torch.zeros(3, device=DEV)
    kw = {}
    if with_loss:
        gen = torch.Generator().manual_seed(100)
        gt = torch.nn.functional.normalize(torch.randn((3, H, W), generator=gen), dim=0).to(DEV)
        mask = (torch.rand((1, H, W), generator=gen) < 0.9).to(DEV)
        kw["language_target"] = (gt, mask)
    train = bench.render(cam, model, bench.Pipe, bg, bench.Opt, **kw)  # the language feature requires grad
    assert train["language_feature_image"].requires_grad
    out_t = {k: v.detach().clone() for k, v in train.items() if torch.is_tensor(v)}
    del train
    with torch.no_grad():
        infer = bench.render(cam, model, bench.Pipe, bg, bench.Opt, **kw)
    torch.cuda.synchronize()
    # the training forward cleared its gradient records; the inference forward wrote no backward state
    assert len(seen) == 2 and seen[0] & _native.FWD_ZERO_GRAD_RECORDS and not seen[0] & _native.FWD_NO_BACKWARD
    assert seen[1] == _native.FWD_NO_BACKWARD
    keys = ["render", "language_feature_image", "radii"] + (["language_l1"] if with_loss else [])
    for k in keys:
        assert torch.equal(infer[k], out_t[k]), k
    assert int((out_t["radii"] > 0).sum()) > 0.3 * P


def test_unfused_rasterizer_under_no_grad_takes_the_inference_flag(monkeypatch):
    """GaussianRasterizer (the unfused autograd Function) with inputs that require grad: under
    torch.no_grad() the forward passes LSR_FWD_NO_BACKWARD, with grad on FWD_ZERO_GRAD_RECORDS, and
    both give the same images."""
    from langsplat_amd.rasterizer import GaussianRasterizer
    seen = _spy_flags(monkeypatch)
    st, inp = scene(P=3000, W=96, H=64, seed=4, scale_range=(0.03, 0.2))
    std, ind = to_device(st, inp, DEV)
    leaves = {k: v.clone().requires_grad_(True) for k, v in ind.items()}
    outs = []
    for grad in (True, False):
        with torch.set_grad_enabled(grad):
            m2 = torch.zeros_like(leaves["means3D"], requires_grad=True)
            c, lg, r = GaussianRasterizer(std)(
                means3D=leaves["means3D"], means2D=m2, opacities=leaves["opacities"], shs=leaves["shs"],
                language_feature_precomp=leaves["language_feature_precomp"], scales=leaves["scales"],
                rotations=leaves["rotations"])
            assert c.requires_grad == grad
            outs.append((c.detach().clone(), lg.detach().clone(), r.clone()))
    torch.cuda.synchronize()
    assert seen == [_native.FWD_ZERO_GRAD_RECORDS, _native.FWD_NO_BACKWARD]
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_backward_after_inference_forward_is_refused_under_debug():
    st, inp = scene(P=800, W=64, H=48, seed=3, scale_range=(0.03, 0.2))
    std, ind = to_device(st._replace(debug=True), inp, DEV)
    args = (ind["means3D"], ind["shs"], None, ind["language_feature_precomp"], ind["opacities"], ind["scales"],
            ind["rotations"], None)
    out = _native.rasterize_gaussians(std, *args, flags=_native.FWD_NO_BACKWARD)
    nr, color, lang, radii, geom, binning, image = out
    ref = _native.rasterize_gaussians(std, *args)
    torch.cuda.synchronize()
    for a, b in zip(out[1:4], ref[1:4]):
        assert torch.equal(a, b)
    with pytest.raises(RuntimeError, match="LSR_FWD_NO_BACKWARD"):
        _native.rasterize_gaussians_backward(std, ind["means3D"], ind["shs"], None, ind["language_feature_precomp"],
                                             ind["scales"], ind["rotations"], None, radii, torch.ones_like(color),
                                             torch.ones_like(lang), nr, geom, binning, image,
                                             opacities=ind["opacities"])
    np.testing.assert_array_equal(radii.cpu().numpy(), ref[3].cpu().numpy())
