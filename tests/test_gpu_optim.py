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
