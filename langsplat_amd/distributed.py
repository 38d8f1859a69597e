"""View-sharded data parallelism: one process per GPU, one camera per rank, one flat gradient
all-reduce per step.

The reference trains on one GPU (utils/general_utils.py:133) with one random view per
iteration (train.py:85-87).  Independent views shard with no data-path exchange; the only
collective is the SUM of the Gaussians' gradients, done here as ONE all-reduce over a single
persistent fp32 bucket whose slices ARE the parameters' .grad tensors (autograd accumulates
straight into it, so there is no pack/unpack copy).  Backend "nccl" is RCCL on ROCm (xGMI);
"gloo" runs the same code on CPU for the tests.
"""
from __future__ import annotations

import os
from typing import Iterable, List

import torch
import torch.distributed as dist

from . import rccl


def init_from_env(backend: str = None):
    """Initialise torch.distributed from torchrun's RANK/WORLD_SIZE/MASTER_* (no-op if WORLD_SIZE<=1)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1 or dist.is_initialized():
        return dist.get_rank() if dist.is_initialized() else 0, world
    if backend is None:  # LSR_DIST_BACKEND=gloo: a rehearsal with several ranks on one GPU
        backend = os.environ.get("LSR_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group(backend=backend)
    return dist.get_rank(), dist.get_world_size()


def collective_capturable(group=None) -> bool:
    """True when the gradient collective is captured into a HIP graph with the step: backend "nccl"
    (RCCL's kernels run on a stream; torch's ProcessGroupNCCL supports stream capture) and
    LSR_GRAPH_COLLECTIVE=1.  gloo reduces on the host and stays an eager call between two graphs.

    The default follows what has run on hardware: with one rank the captured RCCL
    collective is tested (tests/test_gpu_rccl.py) and on; with several ranks it has never run -- a
    one-GPU box cannot host two RCCL ranks (profiles/r06_rccl_two_ranks_one_gpu.txt) -- so there the
    RCCL all-reduce stays an eager launch between the backward and Adam graphs, the form the
    multi-rank gloo runs exercise, unless LSR_GRAPH_COLLECTIVE=1 asks for the captured one."""
    if not (dist.is_available() and dist.is_initialized() and dist.get_backend(group) == "nccl"):
        return False
    default = "1" if dist.get_world_size(group) == 1 else "0"
    return os.environ.get("LSR_GRAPH_COLLECTIVE", default) == "1"


class GradBucket:
    """The trainable parameters' gradients as ONE all-reduce buffer.

    Several parameters (RGB mode: six groups): a flat fp32 buffer whose slices ARE the .grad
    tensors.  Call after the parameters exist and before the first backward; `zero()` clears the
    whole bucket in one memset (optimizer.zero_grad(set_to_none=False) keeps the aliasing; after a
    set_to_none the next all_reduce re-attaches: a fresh .grad is copied into its slice, a missing one
    reads as zeros).

    One parameter (LangSplat's language-feature step, scene/gaussian_model.py:203-217): `direct`
    mode, no buffer of its own.  The .grad tensor autograd leaves (with zero_grad(set_to_none=True)
    it is the rasterizer backward's own output, handed over without a copy) is reduced in place --
    no per-step memset of a bucket and no accumulate-add into it.  A rank whose parameter got no
    gradient this step reduces zeros, so every rank always joins the collective.

    densify_points = P > 0 (RGB mode, train.py:122-126): the bucket also carries the view's
    densification statistics, 2 P floats after the gradients -- per Gaussian ||dL/dmeans2D[:, :2]||
    and the visibility count of this rank's view (stage_densification) -- so the SAME collective
    sums them over the ranks' views, as the reference would accumulate them over that many
    iterations; the MAX of the radii is one more collective over max_radii2D.
    apply_densification then adds the sums into xyz_gradient_accum / denom.
    """

    def __init__(self, params: Iterable[torch.nn.Parameter], densify_points: int = 0):
        self.params: List[torch.Tensor] = [p for p in params if p.requires_grad]
        if not self.params:
            raise ValueError("GradBucket: no trainable parameters")
        for p in self.params:
            if p.dtype != torch.float32:
                raise TypeError("GradBucket expects fp32 parameters")
        self.densify_points = int(densify_points)
        self.direct = len(self.params) == 1 and self.densify_points == 0
        self.flat = None
        self.views = []
        self.stats_norm = self.stats_count = None
        self._divided_by = 1     # what the last all_reduce divided the bucket by (N when averaged)
        self._max_radii = None   # max_radii2D staged for the MAX collective
        if self.direct:
            return
        dev = self.params[0].device
        total = sum(p.numel() for p in self.params)
        self.flat = torch.zeros((total + 2 * self.densify_points,), dtype=torch.float32, device=dev)
        off = 0
        for p in self.params:
            v = self.flat[off:off + p.numel()].view_as(p)
            p.grad = v
            self.views.append(v)
            off += p.numel()
        if self.densify_points:
            P = self.densify_points
            self.stats_norm = self.flat[off:off + P]
            self.stats_count = self.flat[off + P:off + 2 * P]

    def matches(self, params: Iterable[torch.Tensor]) -> bool:
        """True when the bucket was built over exactly these (trainable) tensors, with their current
        sizes.  densify_and_prune and reset_opacity (scene/gaussian_model.py:277-281,326-482) replace
        the parameters: a bucket built before reduces the old tensors' slices."""
        ps = [p for p in params if p.requires_grad]
        if [id(p) for p in ps] != [id(p) for p in self.params]:
            return False
        if not self.direct and any(v.shape != p.shape for p, v in zip(ps, self.views)):
            return False
        return not self.densify_points or self.densify_points == int(ps[0].shape[0])

    @property
    def nbytes(self) -> int:
        return sum(p.numel() for p in self.params) * 4

    def attached(self) -> bool:
        if self.direct:
            g = self.params[0].grad
            return g is not None and g.is_contiguous()
        return all(p.grad is not None and p.grad.data_ptr() == v.data_ptr() for p, v in zip(self.params, self.views))

    def _attach(self):
        """Make every .grad reducible without raising (a rank that raised here would leave the others
        waiting inside the collective)."""
        if self.direct:
            p = self.params[0]
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            elif not p.grad.is_contiguous():
                p.grad = p.grad.contiguous()
            return
        for p, v in zip(self.params, self.views):
            g = p.grad
            if g is not None and g.data_ptr() == v.data_ptr():
                continue
            if g is None:
                v.zero_()
            else:
                v.copy_(g)
            p.grad = v

    def zero(self):
        if self.direct:
            if self.params[0].grad is not None:
                self.params[0].grad.zero_()
            return
        self.flat.zero_()

    def buffer(self) -> torch.Tensor:
        """The tensor the collective reduces (the flat bucket, or the one parameter's .grad)."""
        return self.params[0].grad if self.direct else self.flat

    def stage_densification(self, radii: torch.Tensor, viewspace_grad: torch.Tensor, max_radii2D: torch.Tensor):
        """This rank's view into the bucket's statistics slots (which zero() clears) and into
        max_radii2D (train.py:125-126 for one view).  On a GPU one kernel
        (include/lsr.h lsr_densification_stats); gloo tests on CPU run the reference's torch ops."""
        if not self.densify_points:
            raise RuntimeError("GradBucket: built without densify_points")
        if radii.is_cuda:
            from . import _native
            _native.densification_stats(radii, viewspace_grad, max_radii2D, self.stats_norm, self.stats_count)
        else:
            vis = radii > 0
            max_radii2D[vis] = torch.max(max_radii2D[vis], radii[vis].to(max_radii2D.dtype))
            self.stats_norm[vis] += torch.norm(viewspace_grad[vis, :2], dim=-1)
            self.stats_count[vis] += 1
        self._max_radii = max_radii2D

    def apply_densification(self, xyz_gradient_accum: torch.Tensor, denom: torch.Tensor):
        """xyz_gradient_accum += the ranks' summed norms; denom += their summed visibility counts
        (exact: the counts are integers, recovered from an averaged bucket by rounding)."""
        n = self._divided_by
        if n == 1:
            xyz_gradient_accum.view(-1).add_(self.stats_norm)
            denom.view(-1).add_(self.stats_count)
        else:
            xyz_gradient_accum.view(-1).add_(self.stats_norm * n)
            denom.view(-1).add_(torch.round(self.stats_count * n))

    def all_reduce(self, average: bool = True, group=None, flag: torch.Tensor = None):
        """SUM over ranks (then / world_size when average) -- the one collective of a step (and, with
        staged densification statistics, the MAX of max_radii2D).

        flag: a () int32 device tensor holding 0 or the bits of a positive float -- the rasterizer's
        capacity overflow flag (include/lsr.h lsr_forward_args.overflow: 1.0f when set) -- reduced in
        the SAME collective (coalesced with the gradients), so afterwards it is non-zero on every rank
        as soon as it was on one: every rank then skips the optimizer step on it (optim.Adam
        step(skip=flag)) and the ranks stay identical, as if that iteration's views had been left out.
        Inside a HIP graph capture (RCCL) the collective is captured with the step."""
        if not (dist.is_available() and dist.is_initialized()):
            self._divided_by = 1
            return
        self._attach()
        self._reduce(self.buffer(), average, group, flag)
        if self._max_radii is not None:
            dist.all_reduce(self._max_radii, op=dist.ReduceOp.MAX, group=group)
            self._max_radii = None

    def all_reduce_partials(self, partials: torch.Tensor, average: bool = True, group=None,
                            flag: torch.Tensor = None):
        """The step's collective over a deferred language backward's per-Gaussian partials
        (_native.fused_update(defer=True).partials(), include/lsr.h LSR_BWD_DEFER_TAIL: they end with
        the step's skip word, so no separate flag) instead of the parameter's .grad: the same SUM / AVG
        as all_reduce, before the gradient epilogue, which is linear in them (lsr_language_tail then
        writes the reduced gradient and steps on the reduced skip word).  One parameter (direct mode)
        only."""
        if not self.direct:
            raise RuntimeError("GradBucket.all_reduce_partials: for the one-parameter language step only")
        if not (dist.is_available() and dist.is_initialized()):
            self._divided_by = 1
            return
        self._reduce(partials, average, group, flag)

    def _reduce(self, buf: torch.Tensor, average: bool, group, flag: torch.Tensor):
        world = dist.get_world_size(group)
        nccl = dist.get_backend(group) == "nccl"
        if flag is not None and (flag.dtype != torch.int32 or flag.numel() != 1 or flag.device != buf.device):
            raise ValueError("GradBucket.all_reduce: flag must be a one-element int32 tensor on the bucket's device")
        comm = None
        if nccl and group is None and rccl.direct_enabled(group) and (
                rccl._default is not None or not torch.cuda.is_current_stream_capturing()):
            # RCCL on the caller's stream (langsplat_amd.rccl: no round trip through torch's internal
            # stream); its communicator is built at the first (eager) reduction
            comm = rccl.default_communicator()
        if comm is not None:
            comm.all_reduce([buf] + ([flag.view(torch.float32)] if flag is not None else []),
                            op="avg" if average else "sum")
            self._divided_by = world if average else 1
            return
        # RCCL's ncclAvg: the division is part of the collective (no separate scaling kernel)
        op = dist.ReduceOp.AVG if average and nccl else dist.ReduceOp.SUM
        if flag is None:
            dist.all_reduce(buf, op=op, group=group)
        else:
            if nccl:  # one ncclGroup: one collective launch for both
                with dist._coalescing_manager(group=group):
                    dist.all_reduce(buf, op=op, group=group)
                    dist.all_reduce(flag.view(torch.float32), op=op, group=group)
            else:  # gloo's coalesced all-reduce takes CPU tensors only; it reduces on the host anyway
                dist.all_reduce(buf, op=op, group=group)
                dist.all_reduce(flag.view(torch.float32), op=op, group=group)
        if average and not nccl:
            buf.mul_(1.0 / world)
        self._divided_by = world if average else 1


class UpdateOverlap:
    """The language step's gradient all-reduce and optimiser update on a side stream, overlapped with
    the next view's geometry work (SURVEY.md §8e cost model; VERDICT r02 missing item 5).

    In LangSplat's language step (scene/gaussian_model.py:203-217) every geometry parameter is frozen,
    so the next view's preprocess, depth order and binning -- ~200 us at C3 -- do not depend on the
    update of the language feature.  `update()` enqueues the all-reduce of the step's gradient
    (GradBucket, RCCL on the side stream) and `optimizer.step()` behind the main stream's backward,
    then drops the .grad tensors (zero_grad(set_to_none=True), train.py:138); `forward()` is the
    context for the next render(): its rasterizer forward runs the geometry stages at once and waits
    for the update only before the feature enters the records (include/lsr.h
    lsr_forward_args.language_ready).  Results are identical to the serial step; only the order of
    independent work changes.  `synchronize()` makes the current stream wait for the last update
    (before reading the parameters elsewhere, e.g. a checkpoint)."""

    def __init__(self, bucket: "GradBucket", optimizer, device=None):
        self.bucket = bucket
        self.optimizer = optimizer
        self.side = torch.cuda.Stream(device)
        self.ready = None

    def forward(self):
        from . import _native
        return _native.language_ready(self.ready)

    def update(self, average: bool = True):
        done = torch.cuda.Event()
        done.record()
        self.side.wait_event(done)
        with torch.cuda.stream(self.side):
            for p in self.bucket.params:
                if p.grad is not None:
                    p.grad.record_stream(self.side)  # freed by zero_grad below, still read on the side
            self.bucket.all_reduce(average=average)
            self.optimizer.step()
            ev = torch.cuda.Event()
            ev.record(self.side)
        self.optimizer.zero_grad(set_to_none=True)
        self.ready = ev

    def synchronize(self):
        if self.ready is not None:
            torch.cuda.current_stream().wait_event(self.ready)
