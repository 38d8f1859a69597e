"""langsplat_amd.densify on CPU tensors (no GPU: the statistics are filled by hand): the surgery
keeps every optimizer state aligned with its parameter, and clone / split / prune do what
scene/gaussian_model.py:359-478 does -- clones are exact copies appended after the old Gaussians,
a split Gaussian is replaced by N samples with scale / (0.8 N) and its rotation / colour / opacity,
transparent Gaussians are pruned, the statistics restart at zero."""
import math

import torch

from langsplat_amd.densify import Densifier, quaternion_to_matrix
from langsplat_amd.synthetic import make_gaussians


class _M:
    pass


def _setup(P=400, seed=3):
    g = make_gaussians(P, seed=seed, scale_range=(0.002, 0.05))
    m = _M()
    names = {"xyz": "_xyz", "f_dc": "_features_dc", "f_rest": "_features_rest", "opacity": "_opacity",
             "scaling": "_scaling", "rotation": "_rotation"}
    src = {"xyz": g.xyz, "f_dc": g.features_dc, "f_rest": g.features_rest, "opacity": g.opacity,
           "scaling": g.scaling, "rotation": g.rotation}
    for n, a in names.items():
        setattr(m, a, torch.nn.Parameter(src[n].clone()))
    opt = torch.optim.Adam([{"params": [getattr(m, a)], "lr": 1e-3, "name": n} for n, a in names.items()],
                           lr=0.0, eps=1e-15)
    for a in names.values():
        getattr(m, a).grad = torch.randn_like(getattr(m, a))
    opt.step()  # moments exist
    return m, opt, names


def test_rotation_matrix_is_orthonormal():
    q = torch.randn(50, 4)
    R = quaternion_to_matrix(q)
    torch.testing.assert_close(R @ R.transpose(1, 2), torch.eye(3).expand(50, 3, 3), atol=1e-5, rtol=0)
    torch.testing.assert_close(torch.det(R), torch.ones(50), atol=1e-5, rtol=0)


def test_clone_split_prune_bookkeeping():
    torch.manual_seed(0)
    m, opt, names = _setup()
    P = m._xyz.shape[0]
    d = Densifier(m, opt, percent_dense=0.01)
    d.xyz_gradient_accum = torch.rand((P, 1))
    d.denom = torch.ones((P, 1))
    d.denom[:10] = 0  # never seen: nan -> 0
    d.xyz_gradient_accum[0] = 0.0  # the transparent one below: neither cloned nor split
    grads = d.xyz_gradient_accum / d.denom
    grads[grads.isnan()] = 0.0
    thr = 0.7
    big = torch.exp(m._scaling).max(dim=1).values > 0.01
    clone_sel = (grads.squeeze() >= thr) & ~big
    split_sel = (grads.squeeze() >= thr) & big
    before = {n: getattr(m, a).detach().clone() for n, a in names.items()}
    with torch.no_grad():
        m._opacity[0] = -10.0  # transparent: pruned
    before["opacity"][0] = -10.0
    P1 = d.densify_and_prune(thr, 0.005, 1.0, None)
    nc, ns = int(clone_sel.sum()), int(split_sel.sum())
    assert nc > 0 and ns > 0
    assert P1 == P + nc + ns - 1  # + clones, + 2 per split - the split originals, - the transparent one
    # every optimizer state follows its parameter
    for grp in opt.param_groups:
        p = grp["params"][0]
        assert getattr(m, names[grp["name"]]) is p
        assert opt.state[p]["exp_avg"].shape == p.shape == opt.state[p]["exp_avg_sq"].shape
    # the survivors in order: kept originals (not split, not transparent), clones, split samples
    keep_orig = ~split_sel
    keep_orig[0] = False
    n_keep = int(keep_orig.sum())
    torch.testing.assert_close(m._xyz[:n_keep].detach(), before["xyz"][keep_orig])
    clones = before["xyz"][clone_sel]
    torch.testing.assert_close(m._xyz[n_keep:n_keep + clones.shape[0]].detach(), clones)
    samples = m._scaling[n_keep + clones.shape[0]:].detach()
    assert samples.shape[0] == 2 * ns
    torch.testing.assert_close(samples, (before["scaling"][split_sel] - math.log(1.6)).repeat(2, 1), atol=1e-6,
                               rtol=0)
    torch.testing.assert_close(m._rotation[n_keep + clones.shape[0]:].detach(), before["rotation"][split_sel].repeat(2, 1))
    # the new Gaussians' moments start at zero; the statistics restart
    st = opt.state[m._xyz]
    assert not st["exp_avg"][n_keep:].any() and st["exp_avg"][:n_keep].abs().sum() > 0
    assert d.xyz_gradient_accum.shape == (P1, 1) and not d.xyz_gradient_accum.any() and not d.denom.any()


def _reference_reset_opacity(model, optimizer):
    """scene/gaussian_model.py:277-281 and replace_tensor_to_optimizer :326-339, restated with the
    reference's torch operations (the module itself imports CUDA-only extensions)."""
    op = torch.sigmoid(model._opacity)
    x = torch.min(op, torch.ones_like(op) * 0.01)
    opacities_new = torch.log(x / (1 - x))  # utils/general_utils.py:18-19 inverse_sigmoid
    for group in optimizer.param_groups:
        if group["name"] == "opacity":
            stored_state = optimizer.state.get(group["params"][0], None)
            stored_state["exp_avg"] = torch.zeros_like(opacities_new)
            stored_state["exp_avg_sq"] = torch.zeros_like(opacities_new)
            del optimizer.state[group["params"][0]]
            group["params"][0] = torch.nn.Parameter(opacities_new.requires_grad_(True))
            optimizer.state[group["params"][0]] = stored_state
            model._opacity = group["params"][0]


def test_reset_opacity_matches_the_reference_ops():
    """Densifier.reset_opacity (train.py:132-133): the same raw opacities bit for bit as the
    reference's ops, zero moments, the step count kept, the other groups untouched, and the next
    optimizer step (same iteration, train.py:135-137) leaves the opacity alone (no .grad)."""
    torch.manual_seed(1)
    m, opt, names = _setup(P=300)
    with torch.no_grad():
        m._opacity[:5] = torch.tensor([-8.0, -4.6, -4.5951, 0.0, 3.0]).view(5, 1)  # below, at, above 0.01
    ref_m, ref_opt, _ = _setup(P=300)
    with torch.no_grad():
        for a in names.values():
            getattr(ref_m, a).copy_(getattr(m, a))
    for (pa, pb) in zip([g["params"][0] for g in opt.param_groups], [g["params"][0] for g in ref_opt.param_groups]):
        for k in ("exp_avg", "exp_avg_sq"):
            ref_opt.state[pb][k].copy_(opt.state[pa][k])
    others = {n: getattr(m, a) for n, a in names.items() if n != "opacity"}
    old = m._opacity
    Densifier(m, opt).reset_opacity()
    _reference_reset_opacity(ref_m, ref_opt)
    assert m._opacity is not old and m._opacity.grad is None and m._opacity.requires_grad
    assert torch.equal(m._opacity.detach(), ref_m._opacity.detach())
    assert float(torch.sigmoid(m._opacity.detach()).max()) <= 0.01 + 1e-7
    st = opt.state[m._opacity]
    assert old not in opt.state and not st["exp_avg"].any() and not st["exp_avg_sq"].any()
    assert int(st["step"].item()) == int(ref_opt.state[ref_m._opacity]["step"].item()) == 1
    grp = next(g for g in opt.param_groups if g["name"] == "opacity")
    assert grp["params"][0] is m._opacity
    for n, p in others.items():
        assert getattr(m, names[n]) is p
    before = m._opacity.detach().clone()
    opt.step()  # the same iteration's step: the old tensor's .grad is gone with it
    assert torch.equal(m._opacity.detach(), before)
