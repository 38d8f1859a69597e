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
    """ViewPipeline's order replayed from HIP graphs: every step is one full language step -- view k's
    backward and Adam on one stream, view k+1's forward on the other, its compositing waiting for the
    update -- with no host work between the kernels (langsplat_amd.graph.GraphedStep is the
    unpipelined form).

    The HIP runtime launches one graph's kernels on one queue in capture order, so two branches of a
    single captured graph barely overlap (measured: DESIGN.md §5b).  Here each step is two graph
    launches on two streams: G_bwd (backward + Adam, ending in an external event record of the update)
    and G_fwd (the whole forward of the next view; the rasterizer's wait for the update is an external
    event-wait node, include/lsr.h LSR_FWD_READY_EXTERNAL, so the geometry stages run at once).  A
    backward reads what the previous step's forward wrote, so forwards alternate between two static
    buffer sets (_native.static_buffers: the same addresses at every forward): per set s a forward
    graph G_fwd[s] and a backward graph G_bwd[s].  Host events order the launches: G_bwd[s] after
    G_fwd[s]; G_fwd[s] after the previous G_bwd[s] (its buffers' last reader).  The rasterizer runs
    in capacity mode (capacities from eager warm-up views, with headroom; a view over capacity is
    flagged, check() re-captures).  N = 1: the optimizer is captured (its step count advances on the
    device); a collective is not captured.

        g = PipelinedGraphStep(lambda: render(...)["language_l1"], [gaussians._language_feature], optimizer)
        for it in range(iterations):
            loss = g.replay()   # the loss of the view this step composited (its backward: next step)
        g.synchronize(); g.check(); g.sync()

    forward_fn() runs render() + the loss and returns the loss (no backward).  The graphs own the
    parameters' .grad tensors.  A returned loss is written on the pipeline's forward stream: read it
    after synchronize() (or with .item() after torch.cuda.synchronize())."""

    def __init__(self, forward_fn, params, optimizer, headroom: float = 1.125, warmup: int = 2):
        self.forward_fn = forward_fn
        self.params = [p for p in params]
        self.optimizer = optimizer
        self.headroom = float(headroom)
        self.warmup = int(warmup)
        dev = self.params[0].device
        self.sets = (_native.static_buffers(), _native.static_buffers())
        self.fwd_stream, self.bwd_stream = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        self.overflow = torch.zeros((), dtype=torch.int32, device=dev)
        self.g_fwd = [None, None]
        self.g_bwd = [None, None]
        self.static_loss = [None, None]
        self.ev_fwd = [torch.cuda.Event(), torch.cuda.Event()]
        self.ev_bwd = [torch.cuda.Event(), torch.cuda.Event()]
        self.ev_update = torch.cuda.Event()
        self.next = 0  # the set whose backward the next step runs
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

    def _capture_backward(self, s, loss):
        """G_bwd[s]: the backward of set s's forward (autograd runs it on the forward stream, forked
        into this capture) + the optimizer step, then the update's external event record."""
        A, B = self.fwd_stream, self.bwd_stream
        for p in self.params:
            p.grad = None  # the captured backward assigns its own .grad (no accumulate)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=B):
            fork = torch.cuda.Event()
            fork.record(B)
            A.wait_event(fork)
            loss.backward()
            B.wait_stream(A)
            self.optimizer.step()
            _native.event_record_external(self.ev_update, B)
        self.g_bwd[s] = g

    def _capture_forward(self, s, cap):
        """G_fwd[s]: the next view's forward into set s, its compositing behind the update."""
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=self.fwd_stream):
            with cap, self.sets[s], _native.language_ready(self.ev_update, external=True):
                loss = self.forward_fn()
        self.g_fwd[s] = g
        self.static_loss[s] = loss.detach()  # the set's static loss tensor
        return loss

    def capture(self, min_rendered: int = 0, min_entries: int = 0):
        self._measure(min_rendered, min_entries)
        self.g_fwd, self.g_bwd = [None, None], [None, None]
        self.optimizer.prepare_capture()
        cap = _native.capacity(self.rendered, self.entries, self.overflow)
        A, B = self.fwd_stream, self.bwd_stream
        cur = torch.cuda.current_stream()
        A.wait_stream(cur)
        B.wait_stream(cur)
        # eager forwards allocate both sets at their capacity sizes (no allocation may happen during a
        # capture); set 0's is the prologue, whose backward the first step runs
        with torch.cuda.stream(A):
            for s in (1, 0):
                with cap, self.sets[s]:
                    loss = self.forward_fn()
        self.static_loss[0] = loss.detach()
        self.ev_update.record(B)  # creates the event
        torch.cuda.synchronize()
        self._capture_backward(0, loss)   # backward of the prologue (set 0)
        loss = None
        loss = self._capture_forward(1, cap)
        self._capture_backward(1, loss)
        loss = None
        self._capture_forward(0, cap)     # its autograd graph is not needed: G_bwd[0] holds the kernels
        self.ev_fwd[0].record(A)          # the prologue's forward: the first backward waits for it
        self.next = 0
        self.captures += 1
        return self

    def replay(self) -> torch.Tensor:
        if self.g_fwd[0] is None:
            self.capture()
        s = self.next
        n = 1 - s
        A, B = self.fwd_stream, self.bwd_stream
        B.wait_event(self.ev_fwd[s])          # set s's forward has run
        with torch.cuda.stream(B):
            self.g_bwd[s].replay()            # its backward + Adam (records the update)
        self.ev_bwd[s].record(B)
        A.wait_event(self.ev_bwd[n])          # set n's last reader (the previous step's backward)
        with torch.cuda.stream(A):
            self.g_fwd[n].replay()            # the next view into set n, compositing behind the update
        self.ev_fwd[n].record(A)
        self.next = n
        return self.static_loss[n]

    def synchronize(self):
        """The caller's current stream waits for every step enqueued so far."""
        cur = torch.cuda.current_stream()
        cur.wait_stream(self.fwd_stream)
        cur.wait_stream(self.bwd_stream)

    def sync(self):
        """The optimizer state's step counts from the device (a device-to-host copy)."""
        self.synchronize()
        self.optimizer.sync_steps()

    def check(self) -> bool:
        """True if every replay's view fitted its capacities.  Otherwise re-capture with twice the
        capacities (the over-capacity views were not rasterized) and return False."""
        self.synchronize()
        if int(self.overflow.item()) == 0:
            return True
        self.sync()
        self.overflow.zero_()
        self.capture(2 * self.rendered, 2 * self.entries)
        return False
