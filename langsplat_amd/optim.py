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

Inside a HIP graph capture (langsplat_amd.graph.GraphedStep, langsplat_amd.pipeline) the step count
and the learning rates live on the device (include/lsr.h LSR_ADAM_STEP_WORDS): prepare_capture()
puts them there, every replay of the captured launch advances the count, sync_lr() (the graph
forms call it before each replay) copies changed learning rates there -- so a schedule such as
update_learning_rate(iteration) reaches the replays -- and sync_steps() copies the count back into
state["step"].  The device block is one persistent tensor: a later capture re-seeds it in place, so
an earlier graph that still replays keeps valid pointers.  A captured step may be told to skip
(step(skip=flag): a device int32, the rasterizer's capacity overflow flag): when the flag is set at
run time the update changes nothing and the count does not advance (skipped_steps() counts them).
Eager steps after replays first fetch the device count, and write theirs back.
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
        self._step_dev = None    # int64[ADAM_STEP_WORDS] on the device (graph capture)
        self._dev_ahead = False  # replays may have advanced the device count past state["step"]
        self._lr_order = None    # group index of each table entry of the captured launch
        self._lr_dev = None      # the learning rates last written to the device block
        self._step_offset = {}   # parameter -> its count minus the device count (include/lsr.h, ABI 14)

    def _params_with_grad(self):
        return [p for g in self.param_groups for p in g["params"] if p.grad is not None]

    @torch.no_grad()
    def prepare_capture(self):
        """Before a graph capture of step(): the step count (equal for every parameter, as one
        optimizer steps them together) and the learning rates go to the device block, where the
        captured launch reads (and advances) them."""
        self.sync_steps()
        ps = [p for g in self.param_groups for p in g["params"]]
        for p in ps:  # the state torch's first step creates lazily (no allocation may happen in a capture)
            if len(self.state[p]) == 0:
                self.state[p]["step"] = torch.tensor(0.0)
                self.state[p]["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                self.state[p]["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        dev = ps[0].device
        if self._step_dev is None or self._step_dev.device != dev:
            self._step_dev = torch.zeros((_native.ADAM_STEP_WORDS,), dtype=torch.int64, device=dev)
        self._seed_device_count()
        self._lr_dev = None  # rewritten before the next replay (the table order stays until a capture sets it)
        self._dev_ahead = False

    def _seed_device_count(self):
        """The device count := the largest per-parameter count; every parameter's offset := its count
        minus that (torch's counts differ once a replaced tensor skipped a step, e.g. reset_opacity,
        scene/gaussian_model.py:277-281 + 326-339).  In place: older graphs keep their pointer."""
        counts = {p: int(self.state[p]["step"].item()) for g in self.param_groups for p in g["params"]
                  if len(self.state[p])}
        base = max(counts.values()) if counts else 0
        self._step_offset = {p: c - base for p, c in counts.items()}
        self._step_dev[0].fill_(base)

    def step_offset(self, p) -> int:
        return self._step_offset.get(p, 0)

    @torch.no_grad()
    def sync_steps(self):
        """state["step"] of every parameter from the device count (a device-to-host copy)."""
        if self._step_dev is None or not self._dev_ahead:
            return
        n = int(self._step_dev[0].item())
        for g in self.param_groups:
            for p in g["params"]:
                if len(self.state[p]) and p in self._step_offset:
                    self.state[p]["step"] = torch.tensor(float(n + self._step_offset[p]))
        self._dev_ahead = False

    def skipped_steps(self) -> int:
        """Captured steps skipped so far because their skip flag was set (a device-to-host copy)."""
        return 0 if self._step_dev is None else int(self._step_dev[_native.ADAM_WORD_SKIPPED].item())

    @torch.no_grad()
    def sync_lr(self, stream=None):
        """Before a replay of a captured step: the groups' current learning rates into the device
        block (a small host-to-device copy on the current stream, or on `stream`, only when one
        changed)."""
        if self._step_dev is None:
            return
        self._dev_ahead = True
        if self._lr_order is None:
            return
        lrs = [float(self.param_groups[gi]["lr"]) for gi in self._lr_order]
        if lrs == self._lr_dev:
            return
        src = torch.tensor(lrs, dtype=torch.float64).view(torch.int64).pin_memory()
        w = _native.ADAM_WORD_LR
        if stream is None:
            self._step_dev[w:w + len(lrs)].copy_(src, non_blocking=True)
        else:
            with torch.cuda.stream(stream):
                self._step_dev[w:w + len(lrs)].copy_(src, non_blocking=True)
        self._lr_dev = lrs

    def _register_fused(self, group_index: int):
        """A captured backward applies this optimizer's step to the parameter of that group itself
        (_native.fused_update): the device block's lr word 0 is that group's lr."""
        if not (torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()) or self._step_dev is None:
            raise RuntimeError("langsplat_amd.optim.Adam: a fused update is for a captured step (prepare_capture)")
        self._lr_order, self._lr_dev = [group_index], None

    @torch.no_grad()
    def step(self, closure=None, grad_scale: float = 1.0, skip: torch.Tensor = None, fill=None):
        """One Adam step of every parameter with a gradient; grad_scale multiplies the gradients
        first (1 / N after a SUM all-reduce of N views' gradients; 1.0: as torch.optim.Adam).
        skip (inside a graph capture only): a device int32 flag; a replay that finds it set changes
        nothing (a view the rasterizer did not render, include/lsr.h lsr_adam_multi).
        fill (inside a graph capture only): (record address, raw flags) -- the optimizer's one
        parameter is the language feature, and its updated value also goes into the language slots
        of that forward's render records (include/lsr.h lsr_adam_fill_language: the N > 1 language
        step, whose next composite then needs no fill)."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        capturing = torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
        if capturing and self._step_dev is None:
            raise RuntimeError("langsplat_amd.optim.Adam: call prepare_capture() before capturing step()")
        if skip is not None and not capturing:
            raise RuntimeError("langsplat_amd.optim.Adam: skip= is for a captured step (the host knows eager ones)")
        if skip is not None and (skip.dtype != torch.int32 or skip.numel() != 1 or not skip.is_cuda):
            raise ValueError("langsplat_amd.optim.Adam: skip must be a one-element int32 device tensor")
        if not capturing:
            self.sync_steps()  # replays may have advanced the device count
        fu = _native.fused_update.active()
        fused = fu.param if fu is not None and fu.used and fu.optimizer is self else None
        entries, keep, order = [], [], []
        device = None
        for gi, group in enumerate(self.param_groups):
            beta1, beta2 = group["betas"]
            for p in group["params"]:
                if p.grad is None or p is fused:  # (a fused update stepped it inside the backward)
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
                    float(group["eps"]), self.step_offset(p) if capturing else int(state["step"].item())))
                order.append(gi)
                keep.append(grad)  # a contiguous copy lives until the launch is enqueued (stream order)
        if entries and fused is not None:
            raise RuntimeError("langsplat_amd.optim.Adam: a fused update steps the optimizer's only trainable "
                               "parameter (the language feature of the language step)")
        if fill is not None:
            if not capturing or len(entries) != 1 or entries[0].n % 3 != 0:
                raise RuntimeError("langsplat_amd.optim.Adam: step(fill=) is for a captured step of one "
                                   "P x 3 parameter (the language feature)")
            self._lr_order, self._lr_dev = order, None
            with _native._on_device(device):
                _native._check(_native.load().lsr_adam_fill_language(
                    ctypes.byref(entries[0]), float(grad_scale), ctypes.c_void_p(self._step_dev.data_ptr()),
                    None if skip is None else ctypes.c_void_p(skip.data_ptr()), ctypes.c_void_p(int(fill[0])),
                    int(fill[1]), _native._stream(device)), "lsr_adam_fill_language")
            return loss
        if entries:
            table = (_native.LsrAdamTensor * len(entries))(*entries)
            sd = sk = None
            if capturing:
                # the captured launch reads the learning rates of these groups from the device block;
                # sync_lr() (before every replay) writes them there
                self._lr_order, self._lr_dev = order, None
                sd = ctypes.c_void_p(self._step_dev.data_ptr())
                sk = None if skip is None else ctypes.c_void_p(skip.data_ptr())
            with _native._on_device(device):
                _native._check(_native.load().lsr_adam_multi(len(entries), table, float(grad_scale), sd, sk,
                                                             _native._stream(device)), "lsr_adam_multi")
            if not capturing and self._step_dev is not None:
                # keep the device count (and the offsets) equal to the host's counts: a later replay
                # continues from them
                self._seed_device_count()
        return loss
