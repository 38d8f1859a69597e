"""Adaptive density control of the RGB stage (train.py:120-131; scene/gaussian_model.py:326-482) over
this package's optimizer, gradient bucket and densification-statistics kernel.

LangSplat densifies only in the RGB stage (train.py:121 `if not opt.include_feature`): every
`densification_interval` iterations it clones the small Gaussians whose mean screen-space gradient
exceeds a threshold, splits the large ones into N = 2 samples, and prunes the transparent, the
screen-space-large and the world-space-large ones.  The surgery changes P: every parameter tensor and
its Adam moments are re-allocated (the reference's cat_tensors_to_optimizer / _prune_optimizer), so
anything holding their addresses -- a GradBucket, a captured graph -- must be rebuilt afterwards
(`Densifier.densify_and_prune` returns the new P; langsplat_amd.graph.GraphedStep.capture() again).

The statistics (train.py:124-126, add_densification_stats at :480-482) are one HIP kernel
(_native.densification_stats) or, at N > 1, the GradBucket's slots (distributed.py).  The selection
and the surgery are tensor bookkeeping the reference writes as torch ops; they are restated here as
torch ops on the same tensors and with the same order of operations (so a fixed torch seed gives the
reference's split samples), working on any object with GaussianModel's raw parameter attributes and
on langsplat_amd.optim.Adam or torch.optim.Adam (the same state layout).
"""
from __future__ import annotations

import torch

from . import _native

# the optimizer group names of scene/gaussian_model.py:219-226 and the model attributes they hold
GROUP_ATTR = {"xyz": "_xyz", "f_dc": "_features_dc", "f_rest": "_features_rest", "opacity": "_opacity",
              "scaling": "_scaling", "rotation": "_rotation"}


def quaternion_to_matrix(r: torch.Tensor) -> torch.Tensor:
    """utils/general_utils.py:78-99 build_rotation: (P, 4) unnormalised (w, x, y, z) -> (P, 3, 3)."""
    q = r / torch.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2] + r[:, 3] * r[:, 3])[:, None]
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = torch.zeros((q.size(0), 3, 3), device=r.device, dtype=r.dtype)
    R[:, 0, 0] = 1 - 2 * (y * y + z * z)
    R[:, 0, 1] = 2 * (x * y - w * z)
    R[:, 0, 2] = 2 * (x * z + w * y)
    R[:, 1, 0] = 2 * (x * y + w * z)
    R[:, 1, 1] = 1 - 2 * (x * x + z * z)
    R[:, 1, 2] = 2 * (y * z - w * x)
    R[:, 2, 0] = 2 * (x * z - w * y)
    R[:, 2, 1] = 2 * (y * z + w * x)
    R[:, 2, 2] = 1 - 2 * (x * x + y * y)
    return R


class Densifier:
    """The densification state and surgery of one GaussianModel-like `model` trained by `optimizer`
    (groups named as GROUP_ATTR, one parameter each).  percent_dense: OptimizationParams.percent_dense
    (arguments/__init__.py:87)."""

    def __init__(self, model, optimizer, percent_dense: float = 0.01):
        self.model = model
        self.optimizer = optimizer
        self.percent_dense = float(percent_dense)
        self._reset_stats()

    @property
    def P(self) -> int:
        return int(self.model._xyz.shape[0])

    def _reset_stats(self):
        """training_setup / densification_postfix (scene/gaussian_model.py:198-201, :412-414)."""
        dev = self.model._xyz.device
        self.xyz_gradient_accum = torch.zeros((self.P, 1), device=dev)
        self.denom = torch.zeros((self.P, 1), device=dev)
        self.max_radii2D = torch.zeros((self.P,), device=dev)

    def add_stats(self, radii: torch.Tensor, viewspace_grad: torch.Tensor):
        """train.py:124-126 for one view, one kernel (include/lsr.h lsr_densification_stats)."""
        _native.densification_stats(radii, viewspace_grad, self.max_radii2D, self.xyz_gradient_accum, self.denom)

    # ---- optimizer surgery ------------------------------------------------------------------------
    def _replace(self, make_param, make_moment, names=None):
        """Every group's (or the groups in `names`) parameter p -> make_param(p) and its moments
        m -> make_moment(m) (the state keeps its step count); the model attributes follow."""
        for group in self.optimizer.param_groups:
            if len(group["params"]) != 1 or group.get("name") not in GROUP_ATTR:
                raise ValueError("Densifier: one parameter per group, named as scene/gaussian_model.py:219-226")
            if names is not None and group["name"] not in names:
                continue
            old = group["params"][0]
            state = self.optimizer.state.pop(old, None)
            new = torch.nn.Parameter(make_param(group["name"], old.detach()).requires_grad_(True))
            group["params"][0] = new
            if state is not None:
                state["exp_avg"] = make_moment(state["exp_avg"])
                state["exp_avg_sq"] = make_moment(state["exp_avg_sq"])
                self.optimizer.state[new] = state
            setattr(self.model, GROUP_ATTR[group["name"]], new)

    def _append(self, new: dict):
        """cat_tensors_to_optimizer + densification_postfix (scene/gaussian_model.py:376-414): the new
        Gaussians after the old ones, zero moments for them, statistics reset."""
        self._replace(lambda name, p: torch.cat((p, new[name]), dim=0),
                      lambda m: torch.cat((m, torch.zeros((int(new["xyz"].shape[0]),) + tuple(m.shape[1:]),
                                                          dtype=m.dtype, device=m.device)), dim=0))
        self._reset_stats()

    def _keep(self, keep: torch.Tensor):
        """_prune_optimizer + prune_points (scene/gaussian_model.py:340-374) with keep = ~prune mask."""
        self._replace(lambda name, p: p[keep], lambda m: m[keep])
        self.xyz_gradient_accum = self.xyz_gradient_accum[keep]
        self.denom = self.denom[keep]
        self.max_radii2D = self.max_radii2D[keep]

    def reset_opacity(self):
        """scene/gaussian_model.py:277-281 (train.py:132-133, every opacity_reset_interval): every
        opacity clamped to at most 0.01, as the raw parameter inverse_sigmoid(min(sigmoid(o), 0.01))
        (utils/general_utils.py:18-19), through replace_tensor_to_optimizer (:326-339): a new
        Parameter, both Adam moments zeros, the step count kept.  The new tensor has no .grad, so the
        optimizer step of the same iteration (train.py:135-137) leaves the opacity alone, as in the
        reference.  A captured step holds the old tensor's address: capture it again afterwards."""
        def make(name, p):
            op = torch.sigmoid(p)  # get_opacity (scene/gaussian_model.py:153-155)
            x = torch.min(op, torch.ones_like(op) * 0.01)
            return torch.log(x / (1 - x))
        self._replace(make, torch.zeros_like, names=("opacity",))

    # ---- the three operations ------------------------------------------------------------------------
    def _scales(self):
        return torch.exp(self.model._scaling)

    def densify_and_clone(self, grads, grad_threshold, scene_extent):
        """scene/gaussian_model.py:447-462: copies of the small Gaussians with large gradients."""
        m = self.model
        sel = torch.logical_and(torch.norm(grads, dim=-1) >= grad_threshold,
                                torch.max(self._scales(), dim=1).values <= self.percent_dense * scene_extent)
        self._append({name: getattr(m, attr)[sel].detach() for name, attr in GROUP_ATTR.items()})

    def densify_and_split(self, grads, grad_threshold, scene_extent, N=2):
        """scene/gaussian_model.py:418-445: each large Gaussian with a large gradient becomes N samples
        of itself (positions drawn from it, scales / (0.8 N)); the originals are pruned."""
        m = self.model
        n0 = self.P
        padded = torch.zeros((n0,), device=grads.device)
        padded[:grads.shape[0]] = grads.squeeze()
        sel = torch.logical_and(padded >= grad_threshold,
                                torch.max(self._scales(), dim=1).values > self.percent_dense * scene_extent)
        scales = self._scales()[sel].repeat(N, 1)
        samples = torch.normal(mean=torch.zeros((scales.size(0), 3), device=grads.device), std=scales)
        rots = quaternion_to_matrix(m._rotation[sel].detach()).repeat(N, 1, 1)
        new = {"xyz": torch.bmm(rots, samples.unsqueeze(-1)).squeeze(-1) + m._xyz[sel].detach().repeat(N, 1),
               "scaling": torch.log(scales / (0.8 * N)),
               "rotation": m._rotation[sel].detach().repeat(N, 1),
               "f_dc": m._features_dc[sel].detach().repeat(N, 1, 1),
               "f_rest": m._features_rest[sel].detach().repeat(N, 1, 1),
               "opacity": m._opacity[sel].detach().repeat(N, 1)}
        self._append(new)
        self._keep(~torch.cat((sel, torch.zeros(N * int(sel.sum()), device=sel.device, dtype=torch.bool))))

    def densify_and_prune(self, max_grad, min_opacity, extent, max_screen_size) -> int:
        """scene/gaussian_model.py:464-478 (train.py:128-130); returns the new P."""
        grads = self.xyz_gradient_accum / self.denom
        grads[grads.isnan()] = 0.0
        self.densify_and_clone(grads, max_grad, extent)
        self.densify_and_split(grads, max_grad, extent)
        prune = (torch.sigmoid(self.model._opacity) < min_opacity).squeeze()
        if max_screen_size:
            prune = torch.logical_or(torch.logical_or(prune, self.max_radii2D > max_screen_size),
                                     self._scales().max(dim=1).values > 0.1 * extent)
        self._keep(~prune)
        return self.P
