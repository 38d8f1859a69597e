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
    """Flat fp32 buffer backing the .grad of every trainable parameter.

    Call after the parameters exist and before the first backward.  Keep it by using
    optimizer.zero_grad(set_to_none=False) (a None .grad would detach the parameter from the
    bucket); `zero()` does the same for the whole bucket in one memset.
    """

    def __init__(self, params: Iterable[torch.nn.Parameter]):
        self.params: List[torch.Tensor] = [p for p in params if p.requires_grad]
        if not self.params:
            raise ValueError("GradBucket: no trainable parameters")
        dev = self.params[0].device
        total = sum(p.numel() for p in self.params)
        self.flat = torch.zeros((total,), dtype=torch.float32, device=dev)
        self.views = []
        off = 0
        for p in self.params:
            if p.dtype != torch.float32:
                raise TypeError("GradBucket expects fp32 parameters")
            v = self.flat[off:off + p.numel()].view_as(p)
            p.grad = v
            self.views.append(v)
            off += p.numel()

    @property
    def nbytes(self) -> int:
        return self.flat.numel() * 4

    def attached(self) -> bool:
        return all(p.grad is not None and p.grad.data_ptr() == v.data_ptr() for p, v in zip(self.params, self.views))

    def zero(self):
        self.flat.zero_()

    def all_reduce(self, average: bool = True, group=None):
        """SUM over ranks (then / world_size when average) -- the one collective of a step."""
        if not (dist.is_available() and dist.is_initialized()):
            return
        if not self.attached():
            raise RuntimeError("GradBucket: a parameter's .grad no longer aliases the bucket "
                               "(use zero_grad(set_to_none=False))")
        if average and dist.get_backend(group) == "nccl":
            # RCCL's ncclAvg: the division is part of the collective (no separate scaling kernel)
            dist.all_reduce(self.flat, op=dist.ReduceOp.AVG, group=group)
            return
        dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=group)
        if average:
            self.flat.mul_(1.0 / dist.get_world_size(group))
