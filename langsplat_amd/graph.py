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
count then advances on the device at every replay (sync() copies it back into the optimizer state).
Without, the optimizer runs after each replay on the gradients the graph wrote into the parameters'
.grad tensors.  Either way the graph owns those .grad tensors: do not set them to None.
"""
from __future__ import annotations

from typing import Callable, Iterable

import torch

from . import _native


class GraphedStep:
    def __init__(self, step_fn: Callable[[], torch.Tensor], params: Iterable[torch.Tensor], headroom: float = 1.125,
                 warmup: int = 2, optimizer=None):
        """step_fn: runs render + loss + loss.backward() and returns the loss; params: the tensors
        whose .grad the step produces (the trainable parameters); optimizer: stepped inside the graph."""
        self.step_fn = step_fn
        self.optimizer = optimizer
        self.params = [p for p in params]
        self.headroom = float(headroom)
        self.warmup = int(warmup)
        self.graph = None
        self.static_loss = None
        self.captures = 0
        self.rendered = self.entries = 0
        dev = self.params[0].device
        self.overflow = torch.zeros((), dtype=torch.int32, device=dev)

    def _measure(self, min_rendered=0, min_entries=0):
        """Eager warm-up steps on a side stream (as torch.cuda.graph's docs prescribe); the largest
        per-forward counts they saw, with headroom, become the capacities."""
        _native.LAST_COUNTS.clear()
        side = torch.cuda.Stream(device=self.params[0].device)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(self.warmup):
                for p in self.params:
                    p.grad = None
                self._body()
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
        self.graph = torch.cuda.CUDAGraph()
        with _native.capacity(self.rendered, self.entries, self.overflow):
            with torch.cuda.graph(self.graph):
                self.static_loss = self._body()
        self.captures += 1
        return self

    def _body(self):
        loss = self.step_fn()
        if self.optimizer is not None:
            self.optimizer.step()
        return loss

    def sync(self):
        """The optimizer state's step counts from the device (a device-to-host copy)."""
        if self.optimizer is not None:
            self.optimizer.sync_steps()

    def replay(self) -> torch.Tensor:
        if self.graph is None:
            self.capture()
        self.graph.replay()
        return self.static_loss

    def check(self) -> bool:
        """True if the last replay's views fitted.  Otherwise (a view over capacity: its step was
        not rasterized) re-capture with twice the capacities and return False: run the step again."""
        if int(self.overflow.item()) == 0:
            return True
        # the over-capacity replay was not rasterized, but its optimizer step ran (on zero gradients
        # of that view); the re-capture measures the view again
        self.sync()
        self.capture(2 * self.rendered, 2 * self.entries)
        return False
