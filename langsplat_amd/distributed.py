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


class GradBucket:
    """The trainable parameters' gradients as ONE all-reduce buffer.

    Several parameters (RGB mode: six groups): a flat fp32 buffer whose slices ARE the .grad
    tensors.  Call after the parameters exist and before the first backward, and keep it by using
    optimizer.zero_grad(set_to_none=False) (a None .grad would detach the parameter from the
    bucket); `zero()` clears the whole bucket in one memset.

    One parameter (LangSplat's language-feature step, scene/gaussian_model.py:203-217): `direct`
    mode, no buffer of its own.  The .grad tensor autograd leaves (with zero_grad(set_to_none=True)
    it is the rasterizer backward's own output, handed over without a copy) is contiguous and is
    reduced in place -- no per-step memset of a bucket and no accumulate-add into it.
    """

    def __init__(self, params: Iterable[torch.nn.Parameter]):
        self.params: List[torch.Tensor] = [p for p in params if p.requires_grad]
        if not self.params:
            raise ValueError("GradBucket: no trainable parameters")
        for p in self.params:
            if p.dtype != torch.float32:
                raise TypeError("GradBucket expects fp32 parameters")
        self.direct = len(self.params) == 1
        self.flat = None
        self.views = []
        if self.direct:
            return
        dev = self.params[0].device
        total = sum(p.numel() for p in self.params)
        self.flat = torch.zeros((total,), dtype=torch.float32, device=dev)
        off = 0
        for p in self.params:
            v = self.flat[off:off + p.numel()].view_as(p)
            p.grad = v
            self.views.append(v)
            off += p.numel()

    @property
    def nbytes(self) -> int:
        return sum(p.numel() for p in self.params) * 4

    def attached(self) -> bool:
        if self.direct:
            g = self.params[0].grad
            return g is not None and g.is_contiguous()
        return all(p.grad is not None and p.grad.data_ptr() == v.data_ptr() for p, v in zip(self.params, self.views))

    def zero(self):
        if self.direct:
            if self.params[0].grad is not None:
                self.params[0].grad.zero_()
            return
        self.flat.zero_()

    def buffer(self) -> torch.Tensor:
        """The tensor the collective reduces (the flat bucket, or the one parameter's .grad)."""
        return self.params[0].grad if self.direct else self.flat

    def all_reduce(self, average: bool = True, group=None):
        """SUM over ranks (then / world_size when average) -- the one collective of a step."""
        if not (dist.is_available() and dist.is_initialized()):
            return
        if not self.attached():
            raise RuntimeError("GradBucket: no gradient to reduce -- the parameter's .grad is missing or not "
                               "contiguous (direct mode), or no longer aliases the bucket (use "
                               "zero_grad(set_to_none=False) with several parameters)")
        buf = self.buffer()
        if average and dist.get_backend(group) == "nccl":
            # RCCL's ncclAvg: the division is part of the collective (no separate scaling kernel)
            dist.all_reduce(buf, op=dist.ReduceOp.AVG, group=group)
            return
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
        if average:
            buf.mul_(1.0 / dist.get_world_size(group))
