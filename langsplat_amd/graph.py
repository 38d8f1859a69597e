"""A LangSplat train step captured into a HIP graph (torch.cuda.CUDAGraph over hipGraph).

The step (render() -> loss -> loss.backward(), train.py:92-104) issues about twenty kernels, each
behind Python, autograd and ctypes work on the host, plus -- in the eager rasterizer -- one wait
for the device to learn the view's tile-instance count (include/lsr.h).  Captured once, a replay
submits the whole step as one graph: the host cost per step becomes one replay call and the GPU runs
the kernels back to back, whatever the host's speed.

The capture runs the rasterizer in capacity mode (_native.capacity): its buffers and launch grids
are sized from capacities measured on eager warm-up steps (with headroom), and the device reads the
true counts.  A view over capacity is flagged in `overflow` (not rasterized); `check()` reads the flag
(a device-to-host sync: call it where the loop syncs anyway, e.g. with train.py:108's loss.item())
and, when set, re-captures with larger capacities.

With `optimizer` (langsplat_amd.optim.Adam) its step is captured too, after the backward: its step
count advances on the device at every replay (sync() copies it back into the optimizer state), its
learning rates are copied to the device before each replay (optimizer.sync_lr(): a schedule such as
update_learning_rate, scene/gaussian_model.py:231-241, reaches the replays), and it skips on the
overflow flag: a replay whose view did not fit changes no parameter, moment or step count -- as if
that view had been left out of the sequence.  Without an optimizer, the caller steps
after each replay on the gradients the graph wrote into the parameters' .grad tensors.  Either way
the graph owns those .grad tensors: do not set them to None.

Before capture(), drop the outputs of any eager step (loss, render package): an autograd graph still
alive binds the parameters' AccumulateGrad nodes to the stream it ran on, the captured backward then
waits on that non-capturing stream, and this HIP runtime crashes at the end of the capture
(DESIGN.md §5a).

A sequence of views (train.py:85-87 picks a random camera every iteration): pass view=ViewSlot(...)
and have step_fn render from the slot (it is Camera-like, and carries the language target), then
replay(view=(camera, gt, mask)) copies that view into the slot on the current stream before the
graph runs.  The captured settings point at the slot's tensors, so nothing else changes.
"""
from __future__ import annotations

import os
from typing import Callable, Iterable, Optional

import torch

from . import _native


class ViewSlot:
    """The static per-view inputs of a captured step: contiguous fp32 copies of a Camera's
    world_view_transform / full_proj_transform / camera_center (scene/cameras.py:54-57) and the
    view's language target (gt (3,H,W) fp32, mask (1,H,W) bool: Camera.get_language_feature,
    scene/cameras.py:58-92).  Camera-like (FoVx, FoVy, image_width, image_height and the three
    tensors), so render(slot, ...) reads it as a camera; the captured settings then point at these
    tensors and load() changes the view of the next replay.

    The field of view and the image size are launch arguments of the captured kernels: a view with
    another FoV or size is refused (it needs its own capture)."""

    def __init__(self, camera, gt: Optional[torch.Tensor] = None, mask: Optional[torch.Tensor] = None,
                 device=None):
        dev = torch.device(device) if device is not None else camera.world_view_transform.device
        self.FoVx, self.FoVy = float(camera.FoVx), float(camera.FoVy)
        self.image_width, self.image_height = int(camera.image_width), int(camera.image_height)
        f32 = dict(dtype=torch.float32, device=dev)
        self.world_view_transform = torch.empty((4, 4), **f32)
        self.full_proj_transform = torch.empty((4, 4), **f32)
        self.camera_center = torch.empty((3,), **f32)
        H, W = self.image_height, self.image_width
        self.gt = torch.empty((3, H, W), **f32) if gt is not None else None
        self.mask = torch.empty((1, H, W), dtype=torch.bool, device=dev) if gt is not None else None
        self.load(camera, gt, mask)

    @property
    def language_target(self):
        return (self.gt, self.mask) if self.gt is not None else None

    @staticmethod
    def sources(camera, gt: Optional[torch.Tensor] = None, mask: Optional[torch.Tensor] = None):
        """The device tensors load() reads (for record_stream when it runs on another stream)."""
        ts = [camera.world_view_transform, camera.full_proj_transform, camera.camera_center, gt, mask]
        return [t for t in ts if torch.is_tensor(t) and t.is_cuda]

    def load(self, camera, gt: Optional[torch.Tensor] = None, mask: Optional[torch.Tensor] = None):
        """Copy a view into the slot (on the current stream)."""
        if (float(camera.FoVx), float(camera.FoVy)) != (self.FoVx, self.FoVy) or \
                (int(camera.image_width), int(camera.image_height)) != (self.image_width, self.image_height):
            raise ValueError("ViewSlot: a view with another field of view or image size needs its own capture")
        self.world_view_transform.copy_(camera.world_view_transform)
        self.full_proj_transform.copy_(camera.full_proj_transform)
        self.camera_center.copy_(camera.camera_center)
        if (gt is None) != (self.gt is None):
            raise ValueError("ViewSlot: a language target is given for every view or for none")
        if gt is not None:
            self.gt.copy_(gt.reshape(self.gt.shape))
            m = mask if mask.dtype == torch.bool else mask != 0
            self.mask.copy_(m.reshape(self.mask.shape))
        return self


class _nullctx:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


def _fused_tail_enabled() -> bool:
    """LSR_FUSED_TAIL=0: captured steps keep the separate gradient epilogue and Adam launches
    (measurement knob; include/lsr.h lsr_backward_args.update)."""
    return os.environ.get("LSR_FUSED_TAIL", "1") != "0"


def _as_view(view):
    """(camera, gt, mask), (camera,) or a camera -> (camera, gt, mask)."""
    if isinstance(view, (tuple, list)):
        cam = view[0]
        gt = view[1] if len(view) > 1 else None
        mask = view[2] if len(view) > 2 else None
        return cam, gt, mask
    return view, None, None


class GraphedStep:
    def __init__(self, step_fn: Callable[[], torch.Tensor], params: Iterable[torch.Tensor], headroom: float = 1.125,
                 warmup: int = 2, optimizer=None, view: Optional[ViewSlot] = None):
        """step_fn: runs render + loss + loss.backward() and returns the loss; params: the tensors
        whose .grad the step produces (the trainable parameters); optimizer: stepped inside the graph;
        view: the ViewSlot step_fn renders from (replay(view=...) then changes the view)."""
        self.step_fn = step_fn
        self.optimizer = optimizer
        self.params = [p for p in params]
        self.headroom = float(headroom)
        self.warmup = int(warmup)
        self.view = view
        self.graph = None
        self.static_loss = None
        self.captures = 0
        self.rendered = self.entries = 0
        dev = self.params[0].device
        self.overflow = torch.zeros((), dtype=torch.int32, device=dev)
        self._skipped_base = 0

    def _measure(self, min_rendered=0, min_entries=0):
        """Eager warm-up steps on a side stream (as torch.cuda.graph's docs prescribe); the largest
        per-forward counts they saw, with headroom, become the capacities.  The optimizer is not
        stepped: the warm-up changes no parameter."""
        _native.LAST_COUNTS.clear()
        side = torch.cuda.Stream(device=self.params[0].device)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(self.warmup):
                for p in self.params:
                    p.grad = None
                self.step_fn()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        if not _native.LAST_COUNTS:
            raise RuntimeError("GraphedStep: the step ran no rasterizer forward")
        r = max(v[0] for v in _native.LAST_COUNTS.values())
        e = max(v[1] for v in _native.LAST_COUNTS.values())
        self.rendered = max(int(r * self.headroom) + 1024, int(min_rendered))
        self.entries = max(int(e * self.headroom) + 1024, int(min_entries))

    def capture(self, min_rendered=0, min_entries=0):
        self._measure(min_rendered, min_entries)
        for p in self.params:
            p.grad = None  # the captured backward assigns fresh .grad tensors (no accumulate)
        if self.optimizer is not None:
            self.optimizer.prepare_capture()
            self._skipped_base = self.optimizer.skipped_steps()
        self.graph = torch.cuda.CUDAGraph()
        with _native.capacity(self.rendered, self.entries, self.overflow):
            with torch.cuda.graph(self.graph):
                self.static_loss = self._body()
        self.captures += 1
        return self

    def _body(self):
        if self.optimizer is None:
            return self.step_fn()
        # N = 1, one trainable parameter (the language step): its Adam step runs inside the backward's
        # epilogue pass (_native.fused_update); optimizer.step() then has nothing left to launch
        fuse = _fused_tail_enabled() and len(self.params) == 1
        with _native.fused_update(self.optimizer, self.params[0], skip=self.overflow) if fuse else _nullctx():
            loss = self.step_fn()
            self.optimizer.step(skip=self.overflow)
        return loss

    def sync(self):
        """The optimizer state's step counts from the device (a device-to-host copy)."""
        if self.optimizer is not None:
            self.optimizer.sync_steps()

    def replay(self, view=None) -> torch.Tensor:
        """One captured step; view=(camera, gt, mask) (or a camera) first loads that view into the
        step's ViewSlot on the current stream."""
        if view is not None:
            if self.view is None:
                raise RuntimeError("GraphedStep.replay(view=...) needs the ViewSlot the step renders from")
            self.view.load(*_as_view(view))
        if self.graph is None:
            self.capture()
        if self.optimizer is not None:
            self.optimizer.sync_lr()
        self.graph.replay()
        return self.static_loss

    def check(self) -> bool:
        """True if every replay since the capture fitted its capacities.  Otherwise re-capture with
        twice the capacities and return False.  An over-capacity view was not rasterized; with a
        captured optimizer its replay changed nothing (skipped: run that view again); without one,
        only the LAST replay's flag is seen (call check() after every replay and skip the
        optimizer step yourself)."""
        skipped = 0
        if self.optimizer is not None:
            skipped = self.optimizer.skipped_steps() - self._skipped_base
        if skipped == 0 and int(self.overflow.item()) == 0:
            return True
        self.sync()
        self.capture(2 * self.rendered, 2 * self.entries)
        return False
