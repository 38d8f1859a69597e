"""langsplat_amd.optim.Adam (one HIP kernel per parameter) vs torch.optim.Adam.

Same algorithm, scalar handling and (explicit) FMAs as torch's single-tensor Adam; agreement is
to float rounding: rtol 2e-6 with an absolute floor of 1e-6 x max|value| for entries near zero,
after several steps with a changing learning rate."""
import pytest
import torch

from langsplat_amd.optim import Adam

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("shape", [(1000, 3), (4097,), (33, 1, 3)])
def test_adam_matches_torch(shape):
    g = torch.Generator().manual_seed(sum(shape))
    p0 = torch.randn(shape, generator=g)
    a = p0.clone().to(DEV).requires_grad_(True)
    b = p0.clone().to(DEV).requires_grad_(True)
    mine = Adam([{"params": [a], "lr": 0.01, "name": "x"}], lr=0.0, eps=1e-15)
    ref = torch.optim.Adam([{"params": [b], "lr": 0.01, "name": "x"}], lr=0.0, eps=1e-15, foreach=False)
    for it in range(6):
        gr = torch.randn(shape, generator=g).to(DEV)
        a.grad = gr.clone()
        b.grad = gr.clone()
        for grp in mine.param_groups + ref.param_groups:
            grp["lr"] = 0.01 * (0.7 ** it)  # update_learning_rate-style schedule
        mine.step()
        ref.step()
        sm, sr = mine.state[a], ref.state[b]
        for x, y in ((a.detach(), b.detach()), (sm["exp_avg"], sr["exp_avg"]), (sm["exp_avg_sq"], sr["exp_avg_sq"])):
            torch.testing.assert_close(x, y, rtol=2e-6, atol=1e-6 * float(y.abs().max()))
        assert float(sm["step"]) == float(sr["step"]) == it + 1


# GaussianModel's optimizer surgery, restated from scene/gaussian_model.py (the densification path
# of the RGB stage): _prune_optimizer :341-357 and cat_tensors_to_optimizer :376-397.  They rewrite
# optimizer.state / param_groups directly, so the optimizer must keep torch's state layout.
def _prune_optimizer(opt, mask):
    out = {}
    for group in opt.param_groups:
        stored = opt.state.get(group["params"][0], None)
        if stored is not None:
            stored["exp_avg"] = stored["exp_avg"][mask]
            stored["exp_avg_sq"] = stored["exp_avg_sq"][mask]
            del opt.state[group["params"][0]]
            group["params"][0] = torch.nn.Parameter(group["params"][0][mask].requires_grad_(True))
            opt.state[group["params"][0]] = stored
        else:
            group["params"][0] = torch.nn.Parameter(group["params"][0][mask].requires_grad_(True))
        out[group["name"]] = group["params"][0]
    return out


def _cat_tensors_to_optimizer(opt, tensors):
    out = {}
    for group in opt.param_groups:
        ext = tensors[group["name"]]
        stored = opt.state.get(group["params"][0], None)
        if stored is not None:
            stored["exp_avg"] = torch.cat((stored["exp_avg"], torch.zeros_like(ext)), dim=0)
            stored["exp_avg_sq"] = torch.cat((stored["exp_avg_sq"], torch.zeros_like(ext)), dim=0)
            del opt.state[group["params"][0]]
            group["params"][0] = torch.nn.Parameter(torch.cat((group["params"][0], ext), dim=0).requires_grad_(True))
            opt.state[group["params"][0]] = stored
        else:
            group["params"][0] = torch.nn.Parameter(torch.cat((group["params"][0], ext), dim=0).requires_grad_(True))
        out[group["name"]] = group["params"][0]
    return out


def test_adam_through_densification_surgery():
    """The RGB stage's six parameter groups (scene/gaussian_model.py:219-226) stepped by the HIP Adam
    and by torch.optim.Adam with identical gradients, through a prune and a densify (optimizer state
    masked / extended as the reference does it): parameters and moments stay equal to rounding."""
    g = torch.Generator().manual_seed(5)
    P = 1200
    shapes = {"xyz": (3,), "f_dc": (1, 3), "f_rest": (15, 3), "opacity": (1,), "scaling": (3,), "rotation": (4,)}
    lrs = {"xyz": 1.6e-4, "f_dc": 2.5e-3, "f_rest": 1.25e-4, "opacity": 0.05, "scaling": 5e-3, "rotation": 1e-3}
    init = {k: torch.randn((P,) + s, generator=g) for k, s in shapes.items()}

    def make(cls, **kw):
        ps = {k: torch.nn.Parameter(v.clone().to(DEV)) for k, v in init.items()}
        return cls([{"params": [ps[k]], "lr": lrs[k], "name": k} for k in shapes], lr=0.0, eps=1e-15, **kw)

    mine, ref = make(Adam), make(torch.optim.Adam, foreach=False)
    for it in range(5):
        n = mine.param_groups[0]["params"][0].shape[0]
        for gm, gr in zip(mine.param_groups, ref.param_groups):
            grad = torch.randn(gm["params"][0].shape, generator=g).to(DEV)
            gm["params"][0].grad = grad.clone()
            gr["params"][0].grad = grad.clone()
        mine.step()
        ref.step()
        if it == 1:  # prune_points: keep ~90 %
            keep = (torch.rand((n,), generator=g) > 0.1).to(DEV)
            _prune_optimizer(mine, keep)
            _prune_optimizer(ref, keep)
        if it == 2:  # densify_and_clone: append copies of 100 points
            idx = torch.randint(0, n, (100,), generator=g).to(DEV)
            for opt in (mine, ref):
                _cat_tensors_to_optimizer(opt, {grp["name"]: grp["params"][0].detach()[idx].clone()
                                                for grp in opt.param_groups})
    for gm, gr in zip(mine.param_groups, ref.param_groups):
        a, b = gm["params"][0], gr["params"][0]
        assert a.shape == b.shape and a.shape[0] > 0
        sm, sr = mine.state[a], ref.state[b]
        for x, y in ((a.detach(), b.detach()), (sm["exp_avg"], sr["exp_avg"]), (sm["exp_avg_sq"], sr["exp_avg_sq"])):
            torch.testing.assert_close(x, y, rtol=2e-6, atol=1e-6 * float(y.abs().max()))


def test_adam_one_launch_over_bucket_slices_with_grad_scale():
    """RGB mode's step: the six gradients are slices of one GradBucket (offsets not 16-B aligned:
    the element-wise path beside the float4 one) and a SUM all-reduce's 1 / N is applied inside the
    Adam pass (step(grad_scale=...)); equal to torch.optim.Adam on the scaled gradients."""
    from langsplat_amd.distributed import GradBucket
    g = torch.Generator().manual_seed(6)
    P = 1001
    shapes = {"xyz": (3,), "f_dc": (1, 3), "f_rest": (15, 3), "opacity": (1,), "scaling": (3,), "rotation": (4,)}
    lrs = {"xyz": 1.6e-4, "f_dc": 2.5e-3, "f_rest": 1.25e-4, "opacity": 0.05, "scaling": 5e-3, "rotation": 1e-3}
    init = {k: torch.randn((P,) + s, generator=g) for k, s in shapes.items()}
    mp = {k: torch.nn.Parameter(v.clone().to(DEV)) for k, v in init.items()}
    rp = {k: torch.nn.Parameter(v.clone().to(DEV)) for k, v in init.items()}
    bucket = GradBucket(list(mp.values()))
    mine = Adam([{"params": [mp[k]], "lr": lrs[k], "name": k} for k in shapes], lr=0.0, eps=1e-15)
    ref = torch.optim.Adam([{"params": [rp[k]], "lr": lrs[k], "name": k} for k in shapes], lr=0.0, eps=1e-15,
                           foreach=False)
    scale = 1.0 / 3.0
    for it in range(4):
        bucket.zero()
        for k in shapes:
            grad = torch.randn((P,) + shapes[k], generator=g).to(DEV)
            mp[k].grad.add_(grad)  # autograd accumulates into the bucket slice
            rp[k].grad = grad * scale
        assert bucket.attached()
        mine.step(grad_scale=scale)
        ref.step()
    for k in shapes:
        sm, sr = mine.state[mp[k]], ref.state[rp[k]]
        for x, y in ((mp[k].detach(), rp[k].detach()), (sm["exp_avg"], sr["exp_avg"]),
                     (sm["exp_avg_sq"], sr["exp_avg_sq"])):
            torch.testing.assert_close(x, y, rtol=2e-6, atol=1e-6 * float(y.abs().max()))


def test_densification_stats_kernel_matches_reference_ops():
    """lsr_densification_stats == train.py:125-126 + scene/gaussian_model.py:480-482 as torch ops."""
    from langsplat_amd import _native
    g = torch.Generator().manual_seed(7)
    P = 5003
    radii = torch.randint(-1, 40, (P,), generator=g, dtype=torch.int32).clamp_min(0).to(DEV)
    dm2 = torch.randn((P, 3), generator=g).to(DEV)
    max_r = (torch.rand((P,), generator=g) * 30).to(DEV)
    accum = torch.rand((P, 1), generator=g).to(DEV)
    denom = torch.randint(0, 5, (P, 1), generator=g).float().to(DEV)
    ref = [max_r.clone(), accum.clone(), denom.clone()]
    vis = radii > 0
    ref[0][vis] = torch.max(ref[0][vis], radii[vis])
    ref[1][vis] += torch.norm(dm2[vis, :2], dim=-1, keepdim=True)
    ref[2][vis] += 1
    _native.densification_stats(radii, dm2, max_r, accum, denom)
    torch.testing.assert_close(max_r, ref[0], rtol=0, atol=0)
    torch.testing.assert_close(accum, ref[1], rtol=1e-6, atol=0)
    torch.testing.assert_close(denom, ref[2], rtol=0, atol=0)
    assert vis.any() and (~vis).any()


def test_adam_fill_language_matches_torch_and_fills_records():
    """lsr_adam_fill_language (ABI 15, the N > 1 language update): a captured step(fill=) over the
    raw P x 3 language feature equals torch.optim.Adam on the same (scaled) gradients, step after
    step, writes normalize(feature) -- the activation of gaussian_renderer/__init__.py:87-88 -- into
    the language slots {f0, f1, f2} of every record (3 float4 per Gaussian, slot word b untouched),
    and with the skip flag set changes no parameter or moment but still fills."""
    from langsplat_amd import _native
    from langsplat_amd.graph import graph_capture
    P = 3001
    g = torch.Generator().manual_seed(7)
    p0 = torch.randn((P, 3), generator=g)
    a = p0.clone().to(DEV).requires_grad_(True)
    b = p0.clone().to(DEV).requires_grad_(True)
    mine = Adam([{"params": [a], "lr": 0.0025, "name": "language_feature"}], lr=0.0, eps=1e-15)
    ref = torch.optim.Adam([{"params": [b], "lr": 0.0025, "name": "language_feature"}], lr=0.0, eps=1e-15,
                           foreach=False)
    records = torch.full((P, 12), 7.0, device=DEV)  # {x y cx cy}{cz o r g}{b f0 f1 f2}
    skip = torch.zeros((), dtype=torch.int32, device=DEV)
    grad = torch.zeros((P, 3), device=DEV)
    a.grad = grad
    mine.prepare_capture()
    graph = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side), graph_capture(graph):
        mine.step(grad_scale=0.5, skip=skip, fill=(records.data_ptr(), _native.RAW_LANGUAGE))
    torch.cuda.current_stream().wait_stream(side)
    for it in range(4):
        gr = torch.randn((P, 3), generator=g).to(DEV)
        grad.copy_(gr)
        skip.fill_(1 if it == 2 else 0)
        before = (a.detach().clone(), mine.state[a]["exp_avg"].clone(), mine.state[a]["exp_avg_sq"].clone())
        mine.sync_lr()
        graph.replay()
        torch.cuda.synchronize()
        if it == 2:  # skipped: nothing changes, the records still receive the (unchanged) feature
            assert torch.equal(a.detach(), before[0]) and torch.equal(mine.state[a]["exp_avg"], before[1])
            assert torch.equal(mine.state[a]["exp_avg_sq"], before[2])
        else:
            b.grad = 0.5 * gr
            ref.step()
        torch.testing.assert_close(a.detach(), b.detach(), rtol=2e-6, atol=1e-6 * float(b.detach().abs().max()))
        f = a.detach()
        want = f / (f.norm(dim=-1, keepdim=True) + 1e-9)
        torch.testing.assert_close(records[:, 9:12], want, rtol=1e-6, atol=1e-7)
        assert torch.all(records[:, :9] == 7.0)
    mine.sync_steps()
    assert float(mine.state[a]["step"]) == 3.0 and mine.skipped_steps() == 1
