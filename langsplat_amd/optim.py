"""Adam for the Gaussian parameters on the GPU.

Drop-in for the `torch.optim.Adam(l, lr=0.0, eps=1e-15)` of scene/gaussian_model.py:229 (and
:203-217 in language-feature mode).  Same param_groups ("lr", "betas", "eps", "name" ...), same
per-parameter state keys ("step", "exp_avg", "exp_avg_sq") -- so update_learning_rate
(:231-241) and the densification code that rewrites optimizer state (:326-420) work unchanged --
but every parameter of every group is updated by ONE HIP launch (liblsr.so lsr_adam_multi: one
HBM pass over param / grad / moments per tensor, each tensor with its own group's lr and its own
step count) instead of torch's multi-tensor kernels.  In RGB mode the six gradients are the
slices of the one all-reduced bucket (langsplat_amd.distributed.GradBucket), and a SUM all-reduce's
1 / N is applied inside that same pass (step(grad_scale=...)).  amsgrad, weight decay and maximize
are not used by LangSplat and are not offered.

Inside a HIP graph capture (langsplat_amd.graph.GraphedStep) the step count lives on the device:
prepare_capture() copies it there before the capture, every replay of the captured launch advances
it (include/lsr.h lsr_adam_multi step_dev), and sync_steps() copies it back into state["step"].
"""
from __future__ import annotations

import ctypes

import torch

from . import _native


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        if lr < 0.0 or eps < 0.0 or not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError(f"invalid Adam hyper-parameters lr={lr} betas={betas} eps={eps}")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps))
        self._step_dev = None  # graph capture: (int64 step count + the step's scalars, uint32 ticket) on the device

    def _params_with_grad(self):
        return [p for g in self.param_groups for p in g["params"] if p.grad is not None]

    @torch.no_grad()
    def prepare_capture(self):
        """Before a graph capture of step(): the step count (equal for every parameter, as one
        optimizer steps them together) goes to the device, where the captured launch advances it."""
        ps = [p for g in self.param_groups for p in g["params"]]
        steps = {int(self.state[p]["step"].item()) for p in ps if len(self.state[p])}
        if len(steps) > 1:
            raise RuntimeError("langsplat_amd.optim.Adam: a captured step needs equal step counts")
        missing = [p for p in ps if len(self.state[p]) == 0]
        if missing:
            raise RuntimeError("langsplat_amd.optim.Adam: run one eager step before capturing")
        dev = ps[0].device
        count = torch.zeros((_native.ADAM_STEP_WORDS,), dtype=torch.int64, device=dev)
        count[0] = steps.pop() if steps else 0
        self._step_dev = (count, torch.zeros((1,), dtype=torch.int32, device=dev))

    @torch.no_grad()
    def sync_steps(self):
        """state["step"] of every parameter from the device count (a device-to-host copy)."""
        if self._step_dev is None:
            return
        n = float(self._step_dev[0][0].item())
        for g in self.param_groups:
            for p in g["params"]:
                if len(self.state[p]):
                    self.state[p]["step"] = torch.tensor(n)

    @torch.no_grad()
    def step(self, closure=None, grad_scale: float = 1.0):
        """One Adam step of every parameter with a gradient; grad_scale multiplies the gradients
        first (1 / N after a SUM all-reduce of N views' gradients; 1.0: as torch.optim.Adam)."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        capturing = torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
        if capturing and self._step_dev is None:
            raise RuntimeError("langsplat_amd.optim.Adam: call prepare_capture() before capturing step()")
        entries, keep = [], []
        device = None
        for group in self.param_groups:
            beta1, beta2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.device.type != "cuda" or p.dtype != torch.float32 or not p.is_contiguous():
                    raise RuntimeError("langsplat_amd.optim.Adam: parameters must be contiguous fp32 tensors on a "
                                       "ROCm GPU device (there is no CPU path)")
                if p.grad.is_sparse:
                    raise RuntimeError("langsplat_amd.optim.Adam does not support sparse gradients")
                if device is not None and p.device != device:
                    raise RuntimeError("langsplat_amd.optim.Adam: all parameters must be on one device")
                device = p.device
                grad = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                state = self.state[p]
                if len(state) == 0:
                    state["step"] = torch.tensor(0.0)
                    state["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    state["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                if not capturing:
                    state["step"] += 1
                entries.append(_native.LsrAdamTensor(
                    p.numel(), p.data_ptr(), grad.data_ptr(), state["exp_avg"].data_ptr(),
                    state["exp_avg_sq"].data_ptr(), float(group["lr"]), float(beta1), float(beta2),
                    float(group["eps"]), 0 if capturing else int(state["step"].item())))
                keep.append(grad)  # a contiguous copy lives until the launch is enqueued (stream order)
        if entries:
            table = (_native.LsrAdamTensor * len(entries))(*entries)
            sd = tk = None
            if capturing:
                sd, tk = (ctypes.c_void_p(t.data_ptr()) for t in self._step_dev)
            with _native._on_device(device):
                _native._check(_native.load().lsr_adam_multi(len(entries), table, float(grad_scale), sd, tk,
                                                             _native._stream(device)), "lsr_adam_multi")
        return loss
