"""Software pipeline of LangSplat's language step across views (train.py:76-138 with include_feature).

In the language step every geometry parameter is frozen (scene/gaussian_model.py:203-217): the next
view's preprocess, depth order and binning (~200 us at C3) read nothing the current step's
backward, gradient all-reduce or Adam writes.  Only the language feature changes, and the rasterizer
can take it late (include/lsr.h lsr_forward_args.language_ready: the geometry stages run at once,
the compositing waits for an event).  So the views of consecutive steps run on two alternating HIP
streams:

    stream A:  geometry(k) -> [wait update(k-1)] -> render(k) + loss -> backward(k) -> [all-reduce] -> Adam(k)
    stream B:                                                 geometry(k+1) -> [wait update(k)] -> render(k+1) ...

and view k+1's geometry stages fill the CUs that view k's render backward leaves idle in its tail
(its longest tiles run alone at the end) and that the all-reduce and Adam leave idle.  Every step
computes exactly what the serial loop computes, in the same order per parameter: view k+1 composites
with the feature Adam(k) wrote.  Autograd runs a node's backward on its forward's stream, so the
backward of view k stays on stream A without further plumbing.

    pipe = ViewPipeline(optimizer)                  # optimizer: langsplat_amd.optim.Adam (or torch's)
    for cam in views:
        with pipe.step():
            loss = render(cam, gaussians, pipe_params, bg, opt, language_target=(gt, mask))["language_l1"]
            loss.backward()
            pipe.update()                           # [all-reduce,] Adam, zero_grad(set_to_none=True)
    pipe.synchronize()                              # before reading the parameters on another stream

A step's tensors (the loss, the images) live on that step's stream: `.item()` is safe anywhere;
using them in device work on another stream needs `pipe.synchronize()` first.  Do not keep a step's
loss (its autograd graph) alive into the next step: the parameters' AccumulateGrad nodes would then
stay bound to the previous step's stream.
"""
from __future__ import annotations

import contextlib

import torch

from . import _native


class ViewPipeline:
    def __init__(self, optimizer, bucket=None, device=None):
        """optimizer: steps the trainable parameters; bucket: a langsplat_amd.distributed.GradBucket
        whose all-reduce precedes the optimizer at N > 1 (None at N = 1)."""
        self.optimizer = optimizer
        self.bucket = bucket
        self.streams = (torch.cuda.Stream(device), torch.cuda.Stream(device))
        self.k = 0
        self.ready = None       # event after the last update (the next forward waits for it)
        self._in_step = False

    @contextlib.contextmanager
    def step(self):
        """One view's step on this step's stream; its rasterizer forward defers the language feature
        until the previous step's update has landed."""
        if self._in_step:
            raise RuntimeError("ViewPipeline.step() blocks do not nest")
        s = self.streams[self.k & 1]
        # whatever the caller enqueued on its own stream before this step (parameter surgery,
        # learning-rate changes done on the device, ...) happens first
        s.wait_stream(torch.cuda.current_stream())
        self._in_step = True
        try:
            with torch.cuda.stream(s), _native.language_ready(self.ready):
                yield s
        finally:
            self._in_step = False
            self.k += 1

    def update(self, average: bool = True):
        """Inside step(), after loss.backward(): the gradient all-reduce (N > 1), the optimizer step and
        zero_grad, on this step's stream; the next step's compositing waits for them."""
        if not self._in_step:
            raise RuntimeError("ViewPipeline.update() belongs inside a step() block")
        if self.bucket is not None:
            self.bucket.all_reduce(average=average)
        self.optimizer.step()
        if self.bucket is not None and not self.bucket.direct:
            self.bucket.zero()
        else:
            self.optimizer.zero_grad(set_to_none=True)
        ev = torch.cuda.Event()
        ev.record()
        self.ready = ev

    def synchronize(self):
        """The caller's current stream waits for every step enqueued so far."""
        cur = torch.cuda.current_stream()
        for s in self.streams:
            cur.wait_stream(s)


class PipelinedGraphStep:
    """ViewPipeline's order captured into HIP graphs: every replay is one full language step --
    view k's backward and Adam on one branch, view k+1's geometry stages on the other, joined before
    view k+1's compositing -- with no host work between the kernels (langsplat_amd.graph.GraphedStep
    is the unpipelined form).

    The HIP runtime launches a graph's kernels on one queue in capture order, so the two branches
    overlap only where independent kernels meet (measured); the eager ViewPipeline
    overlaps more when the host keeps ahead.  (Two graphs on two streams joined by external event
    nodes would overlap fully, but this runtime refuses hipEventRecordExternal in a capture and
    crashes on an external wait.)

    A replay's backward reads what the PREVIOUS replay's forward wrote, so the forwards alternate
    between two static buffer sets (_native.static_buffers: the same addresses at every forward) and
    two graphs, G1 (backward of set 0, forward into set 1) and G0 (the reverse), replayed in turn.
    The rasterizer runs in capacity mode (capacities from eager warm-up views, with headroom; a view
    over capacity is flagged, check() re-captures).  N = 1: the optimizer is captured (its step count
    advances on the device); a collective is not captured.

        g = PipelinedGraphStep(lambda: render(...)["language_l1"], [gaussians._language_feature], optimizer)
        for it in range(iterations):
            loss = g.replay()   # the loss of the view this replay composited (its backward: next replay)
        g.check(); g.sync()

    forward_fn() runs render() + the loss and returns the loss (no backward).  The graphs own the
    parameters' .grad tensors."""

    def __init__(self, forward_fn, params, optimizer, headroom: float = 1.125, warmup: int = 2):
        self.forward_fn = forward_fn
        self.params = [p for p in params]
        self.optimizer = optimizer
        self.headroom = float(headroom)
        self.warmup = int(warmup)
        dev = self.params[0].device
        self.sets = (_native.static_buffers(), _native.static_buffers())
        self.streams = (torch.cuda.Stream(dev), torch.cuda.Stream(dev))
        self.overflow = torch.zeros((), dtype=torch.int32, device=dev)
        self.graphs = [None, None]
        self.static_loss = [None, None]
        self.next = 1
        self.captures = 0
        self.rendered = self.entries = 0

    def _measure(self, min_rendered, min_entries):
        _native.LAST_COUNTS.clear()
        side = torch.cuda.Stream(device=self.params[0].device)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(self.warmup):
                for p in self.params:
                    p.grad = None
                self.forward_fn().backward()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        if not _native.LAST_COUNTS:
            raise RuntimeError("PipelinedGraphStep: forward_fn ran no rasterizer forward")
        r = max(v[0] for v in _native.LAST_COUNTS.values())
        e = max(v[1] for v in _native.LAST_COUNTS.values())
        self.rendered = max(int(r * self.headroom) + 1024, int(min_rendered))
        self.entries = max(int(e * self.headroom) + 1024, int(min_entries))

    def capture(self, min_rendered: int = 0, min_entries: int = 0):
        self._measure(min_rendered, min_entries)
        self.graphs = [None, None]
        self.static_loss = [None, None]
        self.optimizer.prepare_capture()
        cap = _native.capacity(self.rendered, self.entries, self.overflow)
        cur = torch.cuda.current_stream()
        for s in self.streams:
            s.wait_stream(cur)
        # eager forwards allocate both sets at their capacity sizes (no allocation may happen during a
        # capture); set 0's is the prologue: the first replay (G1) runs its backward
        for parity in (1, 0):
            with torch.cuda.stream(self.streams[parity]), cap, self.sets[parity]:
                prev = self.forward_fn()
        pool = torch.cuda.graph_pool_handle()
        for parity in (1, 0):
            bwd_s, fwd_s = self.streams[1 - parity], self.streams[parity]
            for p in self.params:
                p.grad = None  # the captured backward assigns its own .grad (no accumulate)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool, stream=bwd_s):
                fork = torch.cuda.Event()
                fork.record(bwd_s)
                fwd_s.wait_event(fork)
                prev.backward()       # on bwd_s: autograd runs it on its forward's stream
                prev = None           # release the autograd graph (and its AccumulateGrad nodes)
                self.optimizer.step()
                ready = torch.cuda.Event()
                ready.record(bwd_s)
                with torch.cuda.stream(fwd_s), cap, self.sets[parity], _native.language_ready(ready):
                    loss = self.forward_fn()
                bwd_s.wait_stream(fwd_s)
            self.graphs[parity] = g
            self.static_loss[parity] = loss.detach()  # the set's static loss tensor
            prev = loss
            loss = None
        # G0's forward (set 0) is never backwarded by Python: the graphs hold the kernels it captured
        # (replays change the views' data in place, e.g. a camera's matrices copied into the tensors
        # the captured settings point at; the graphs' launches stay the same)
        del prev
        cur.wait_stream(self.streams[0])
        cur.wait_stream(self.streams[1])
        self.next = 1
        self.captures += 1
        return self

    def replay(self) -> torch.Tensor:
        if self.graphs[0] is None:
            self.capture()
        k = self.next
        self.graphs[k].replay()
        self.next = 1 - k
        return self.static_loss[k]

    def synchronize(self):
        """A replay runs on the caller's current stream (its branches join before it ends): nothing
        to wait for beyond stream order."""

    def sync(self):
        """The optimizer state's step counts from the device (a device-to-host copy)."""
        self.optimizer.sync_steps()

    def check(self) -> bool:
        """True if every replay's view fitted its capacities.  Otherwise re-capture with twice the
        capacities (the over-capacity views were not rasterized) and return False."""
        if int(self.overflow.item()) == 0:
            return True
        self.sync()
        self.overflow.zero_()
        self.capture(2 * self.rendered, 2 * self.entries)
        return False
