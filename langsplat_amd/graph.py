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

Stale autograd state.  LangSplat's train loop keeps the previous iteration's render package and loss
alive (train.py:92-108).  Such a graph holds the parameters' AccumulateGrad nodes, each bound to the
stream it was created on; a capture that reused them would make the captured backward wait on that
non-capturing stream (torch warns "AccumulateGrad node's stream does not match"; this HIP runtime
then crashes at the end of the capture).  capture() therefore first releases every
parameter's cached node (release_stale_accumulators, csrc/lsr_autograd.cpp): the warm-up and the
capture create their own, on their own streams, and the caller's old graph keeps its node.  `params`
must list every leaf the step differentiates.  The captured graph's own autograd state is not kept
(the static loss is detached), so eager steps after a capture start clean as well.

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


def graph_capture(graph, stream=None):
    """torch.cuda.graph in thread-local capture mode.  In the default (global) mode an unsafe HIP call
    from ANY thread invalidates the capture, and at N > 1 the process group's watchdog thread polls
    the events of the eager warm-up collective while the step is captured (seen as
    hipErrorStreamCaptureInvalidated at capture_end of a re-capture, then an abort from the
    watchdog); the captures here make no unsafe call themselves."""
    return torch.cuda.graph(graph, stream=stream, capture_error_mode="thread_local")


def release_stale_accumulators(params) -> int:
    """Make every parameter forget its cached AccumulateGrad node (a node a still-alive autograd graph
    holds, bound to the stream that graph ran on), so the next graph creates a fresh one on its own
    stream.  Returns how many parameters had one.  Call before a capture."""
    helper = _native.autograd_helper()
    n = 0
    for p in params:
        if p.requires_grad and p.is_leaf and helper.release_accumulator(p):
            n += 1
        if helper.accumulator_stream(p) is not None:
            raise RuntimeError("release_stale_accumulators: a parameter's AccumulateGrad node is still cached")
    return n


def capture_key(model, optimizer, params):
    """What a captured step bakes in that the reference's train loop changes between iterations:
    the active SH degree (train.py:81-82 oneupSHdegree, scene/gaussian_model.py:166-168: a kernel
    argument of the captured preprocess) and the parameter tensors themselves (densify_and_prune and
    reset_opacity, train.py:128-133, replace them: the graph holds the old addresses).  A replay whose
    key differs from its capture's re-captures first."""
    deg = getattr(model, "active_sh_degree", None) if model is not None else None
    ps = [p for g in optimizer.param_groups for p in g["params"]] if optimizer is not None else list(params)
    return (deg, tuple((id(p), p.data_ptr(), tuple(p.shape)) for p in ps))


def current_params(optimizer, params):
    """The tensors a captured step differentiates: the optimizer's current trainable parameters
    (densification and reset_opacity replace them in its groups), else the given list."""
    if optimizer is None:
        return list(params)
    return [p for g in optimizer.param_groups for p in g["params"] if p.requires_grad]


def resolve_bucket(bucket, factory, params):
    """The gradient bucket a (re-)capture reduces: `bucket` while it was built over `params`;
    otherwise a fresh one from factory(params) -- or an error, since a stale bucket would reduce the
    replaced tensors' slices and leave the new gradients un-averaged (ranks drifting apart)."""
    if bucket is None or bucket.matches(params):
        return bucket
    if factory is None:
        raise RuntimeError("the parameters were replaced since the GradBucket was built (densification, "
                           "reset_opacity): pass bucket_factory= to rebuild it at the re-capture")
    nb = factory(params)
    if not nb.matches(params):
        raise RuntimeError("bucket_factory(params) returned a bucket over other tensors")
    return nb


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
                 warmup: int = 2, optimizer=None, view: Optional[ViewSlot] = None, model=None, bucket=None,
                 bucket_factory=None):
        """step_fn: runs render + loss + loss.backward() and returns the loss; params: the tensors
        whose .grad the step produces (the trainable parameters); optimizer: stepped inside the graph;
        view: the ViewSlot step_fn renders from (replay(view=...) then changes the view); model: the
        GaussianModel step_fn renders (its active_sh_degree is part of the capture key, capture_key).
        With an optimizer, a replay after its parameters were replaced (densification, reset_opacity)
        re-captures over the optimizer's current parameters.  bucket (N > 1, with an optimizer): a
        langsplat_amd.distributed.GradBucket whose all-reduce -- carrying the overflow flag, so every
        rank skips when one view overflowed -- runs between the backward and Adam: inside the graph
        with RCCL, between two graphs with gloo.  A re-capture after the parameters were replaced
        rebuilds the bucket with bucket_factory(params) (`self.bucket` is then the new one; a step_fn
        that stages densification statistics reads it from there) and raises without a factory."""
        if bucket is not None and optimizer is None:
            raise ValueError("GraphedStep: a bucket is reduced before the captured optimizer step")
        self.bucket = bucket
        self.bucket_factory = bucket_factory
        self.graph_adam = None
        self.step_fn = step_fn
        self.model = model
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
        # the optimizer's current tensors (densification replaces them), and a bucket over those
        self.params = current_params(self.optimizer, self.params)
        self.bucket = resolve_bucket(self.bucket, self.bucket_factory, self.params)
        self.key = capture_key(self.model, self.optimizer, self.params)
        self.stale_released = release_stale_accumulators(self.params)  # the caller's held graphs (module doc)
        self._measure(min_rendered, min_entries)
        for p in self.params:
            p.grad = None  # the captured backward assigns fresh .grad tensors (no accumulate)
        if self.optimizer is not None:
            self.optimizer.prepare_capture()
            self._skipped_base = self.optimizer.skipped_steps()
        self.graph = self.graph_adam = None  # an earlier graph's pool goes before the new capture allocates
        self.static_loss = None
        from .distributed import collective_capturable
        self._coll_in_graph = self.bucket is not None and collective_capturable()
        if self._coll_in_graph:  # the communicator exists before the capture (its creation is not capturable)
            self.bucket.all_reduce(average=True, flag=torch.zeros_like(self.overflow))
            for p in self.params:
                p.grad = None
        graph = torch.cuda.CUDAGraph()
        with _native.capacity(self.rendered, self.entries, self.overflow):
            with graph_capture(graph):
                # detached: the captured step's autograd graph (and its AccumulateGrad nodes, bound
                # to the capture stream) is not kept alive past the capture
                self.static_loss = self._body().detach()
        if self.bucket is not None and not self._coll_in_graph:  # gloo: Adam in a graph of its own
            # the graph's gradient tensors; Adam reads what the all-reduce leaves in .grad (the bucket's
            # slices in flat mode, these tensors in direct mode)
            self._graph_grads = [p.grad for p in self.params]
            self.bucket._attach()
            g = torch.cuda.CUDAGraph()
            with graph_capture(g):
                self.optimizer.step(skip=self.overflow)
            self.graph_adam = g
        self.graph = graph
        self.captures += 1
        return self

    def _body(self):
        if self.optimizer is None:
            return self.step_fn()
        # N = 1, one trainable parameter (the language step): its Adam step runs inside the backward's
        # epilogue pass (_native.fused_update); optimizer.step() then has nothing left to launch
        fuse = _fused_tail_enabled() and len(self.params) == 1 and self.bucket is None
        with _native.fused_update(self.optimizer, self.params[0], skip=self.overflow) if fuse else _nullctx():
            loss = self.step_fn()
            if self.bucket is not None:
                if not self._coll_in_graph:
                    return loss  # gloo: the all-reduce and Adam follow the graph (replay)
                self.bucket.all_reduce(average=True, flag=self.overflow)
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
        elif capture_key(self.model, self.optimizer, self.params) != self.key:
            # an SH-degree step or replaced parameters since the capture: capture the step as it is now
            self.sync()
            self.capture(self.rendered, self.entries)
        if self.optimizer is not None:
            self.optimizer.sync_lr()
        self.graph.replay()
        if self.graph_adam is not None:
            for p, g in zip(self.params, self._graph_grads):
                p.grad = g
            self.bucket.all_reduce(average=True, flag=self.overflow)
            self.graph_adam.replay()
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
