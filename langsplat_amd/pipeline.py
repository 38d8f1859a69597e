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
import os

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
    """ViewPipeline's order as HIP graphs on two streams: view k+1's geometry stages run on stream B
    while view k's compositing, loss, backward and Adam run on stream A, with no host work between
    the kernels (langsplat_amd.graph.GraphedStep is the unpipelined form).

    The rasterizer forward is split in two calls (include/lsr.h lsr_forward_args.phase, capacity
    mode): the geometry half (preprocess, depth order, binning; the language feature deferred) and
    the composite half (the feature into the records, compositing, fused loss).  Per static buffer
    set p (_native.static_buffers: the same addresses at every forward) two graphs are captured:

        G_geo[p]:  the geometry half of the view, into set p                  (stream B)
        G_comp[p]: the composite half of set p and the loss                     (stream A)
        G_step[p]: loss.backward() + optimizer.step()                           (stream A)

    and replay k runs (p = k % 2, q = 1 - p):

        stream A:  wait geo[p] -> G_comp[p] -> record comp[p] -> G_step[p] -> record step[p]
        stream B:  wait step[q] -> G_geo[q] -> record geo[q]      (set q is free once step q ran)

    Beside the compositing kernels, which hold every CU slot, the geometry's short launches stretch
    (kernel trace: publish 5 -> 60 us), but starting it only after the compositing (LSR_PG_GEO=fwd)
    measured slower: 0.54 against 0.49 ms per step at C3.

    so a replay is one full language step (the loss it returns is that of the view it composited and
    updated from) and the next view's geometry overlaps it.  Two graphs on two streams are separate
    queues: unlike one graph with two branches (which this HIP runtime launches on one queue in
    capture order), they run concurrently.  The geometry reads nothing the step
    writes (the language step freezes the geometry, scene/gaussian_model.py:203-217); the step's
    feature fill reads what the previous step's Adam wrote (stream A order).

    The rasterizer runs in capacity mode (capacities from eager warm-up views, with headroom; a view
    over capacity is flagged per set, check() re-captures).  N = 1: the optimizer is captured (its
    step count advances on the device); a collective is not captured.

        g = PipelinedGraphStep(lambda: render(...)["language_l1"], [gaussians._language_feature], optimizer)
        for it in range(iterations):
            loss = g.replay()   # this replay's view's loss (on the caller's stream after the replay)
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
        # A: step, B: geometry.  (Stream priorities measured worse: a high-priority geometry stream
        # 0.82 ms per step, a high-priority step stream 0.57, none 0.48; LSR_PG_PRIO=geo / step)
        prio = os.environ.get("LSR_PG_PRIO", "none")
        # the next view's geometry starts with the step ("start") or after this view's compositing
        # ("fwd": beside the backward and Adam only); measured C3: start 0.49, fwd 0.54 ms per step
        self.geo_after_fwd = os.environ.get("LSR_PG_GEO", "start") == "fwd"
        self.streams = (torch.cuda.Stream(dev, priority=-1 if prio == "step" else 0),
                        torch.cuda.Stream(dev, priority=-1 if prio == "geo" else 0))
        self.overflow = (torch.zeros((), dtype=torch.int32, device=dev),
                         torch.zeros((), dtype=torch.int32, device=dev))
        self.g_geo = [None, None]
        self.g_comp = [None, None]
        self.g_step = [None, None]
        self.static_loss = [None, None]
        self.ev_geo = [None, None]
        self.ev_comp = [None, None]
        self.ev_step = [None, None]
        self.next = 0
        self.primed = False
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
        for p in self.params:
            p.grad = None
        if not _native.LAST_COUNTS:
            raise RuntimeError("PipelinedGraphStep: forward_fn ran no rasterizer forward")
        r = max(v[0] for v in _native.LAST_COUNTS.values())
        e = max(v[1] for v in _native.LAST_COUNTS.values())
        self.rendered = max(int(r * self.headroom) + 1024, int(min_rendered))
        self.entries = max(int(e * self.headroom) + 1024, int(min_entries))

    def capture(self, min_rendered: int = 0, min_entries: int = 0):
        self._measure(min_rendered, min_entries)
        self.g_geo = [None, None]
        self.g_comp = [None, None]
        self.g_step = [None, None]
        self.static_loss = [None, None]
        self.optimizer.prepare_capture()
        cur = torch.cuda.current_stream()
        sa, sb = self.streams
        for s in self.streams:
            s.wait_stream(cur)
        caps = [_native.capacity(self.rendered, self.entries, self.overflow[p]) for p in (0, 1)]
        # eager forwards allocate both sets at their capacity sizes (no allocation may happen during
        # a capture); nothing is updated
        for p in (0, 1):
            with torch.cuda.stream(sa), caps[p], self.sets[p]:
                self.forward_fn()
        sb.wait_stream(sa)
        for p in (0, 1):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=sb), caps[p], self.sets[p], \
                    _native.forward_phase(_native.forward_phase.GEOMETRY):
                self.forward_fn()  # its outputs are written by the composite half
            self.g_geo[p] = g
            for q in self.params:
                q.grad = None  # the captured backward assigns its own .grad (no accumulate)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=sa), caps[p], self.sets[p], \
                    _native.forward_phase(_native.forward_phase.COMPOSITE):
                loss = self.forward_fn()
            self.g_comp[p] = g
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=sa):  # the backward runs on its forward's stream (sa)
                loss.backward()
                self.optimizer.step()
            self.g_step[p] = g
            self.static_loss[p] = loss.detach()  # the set's static loss tensor
            del loss
        cur.wait_stream(sa)
        cur.wait_stream(sb)
        self.ev_geo = [torch.cuda.Event(), torch.cuda.Event()]
        self.ev_comp = [torch.cuda.Event(), torch.cuda.Event()]
        self.ev_step = [torch.cuda.Event(), torch.cuda.Event()]
        self.next = 0
        self.primed = False
        self.captures += 1
        return self

    def replay(self) -> torch.Tensor:
        if self.g_step[0] is None:
            self.capture()
        sa, sb = self.streams
        cur = torch.cuda.current_stream()
        p = self.next
        q = 1 - p
        if not self.primed:  # the first view's geometry (set p is free: nothing ran since the capture)
            sb.wait_stream(cur)
            with torch.cuda.stream(sb):
                self.g_geo[p].replay()
            self.ev_geo[p].record(sb)
            self.primed = True
        # the caller's earlier work (e.g. a learning-rate change on the device) precedes the step
        sa.wait_stream(cur)
        sa.wait_event(self.ev_geo[p])
        with torch.cuda.stream(sa):
            self.g_comp[p].replay()
            self.ev_comp[p].record(sa)
            self.g_step[p].replay()
        self.ev_step[p].record(sa)
        # the next view's geometry into set q, once the step that last read set q has run
        sb.wait_event(self.ev_step[q])  # (an event never recorded: no wait)
        if self.geo_after_fwd:
            sb.wait_event(self.ev_comp[p])
        with torch.cuda.stream(sb):
            self.g_geo[q].replay()
        self.ev_geo[q].record(sb)
        cur.wait_event(self.ev_step[p])
        self.next = q
        return self.static_loss[p]

    def synchronize(self):
        """The caller's current stream waits for every replay enqueued so far (both streams)."""
        cur = torch.cuda.current_stream()
        for s in self.streams:
            cur.wait_stream(s)

    def sync(self):
        """The optimizer state's step counts from the device (a device-to-host copy)."""
        self.optimizer.sync_steps()

    def check(self) -> bool:
        """True if every replay's view fitted its capacities.  Otherwise re-capture with twice the
        capacities (the over-capacity views were not rasterized) and return False."""
        self.synchronize()
        if int(self.overflow[0].item()) == 0 and int(self.overflow[1].item()) == 0:
            return True
        self.sync()
        for o in self.overflow:
            o.zero_()
        self.capture(2 * self.rendered, 2 * self.entries)
        return False
