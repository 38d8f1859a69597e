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
from .distributed import collective_capturable
from .graph import (_as_view, _fused_tail_enabled, _nullctx, capture_key, current_params, graph_capture,
                    release_stale_accumulators, resolve_bucket)


# LSR_PG_NATIVE_LAUNCH=0: every replay through torch's stream context and CUDAGraph.replay() (A/B)
_NATIVE_LAUNCH = os.environ.get("LSR_PG_NATIVE_LAUNCH", "1") != "0"

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
    """ViewPipeline's order as HIP graphs on two streams: the geometry stages of a later view run on
    stream B while view k's compositing, loss, backward and Adam run on stream A, with no host work
    between the kernels (langsplat_amd.graph.GraphedStep is the unpipelined form).

    The rasterizer forward is split in two calls (include/lsr.h lsr_forward_args.phase, capacity
    mode): the geometry half (preprocess, depth order, binning; the language feature deferred) and
    the composite half (the feature into the records, compositing, fused loss).  Per static buffer
    set p (_native.static_buffers: the same addresses at every forward; S sets, default 3) the graphs

        G_geo[p]:  the geometry half of the view, into set p                  (stream B)
        G_comp[p]: the composite half of set p and the loss, then loss.backward() and
                   optimizer.step(skip=overflow[p])                             (stream A)
                   (N > 1: the bucket's all-reduce between the backward and Adam -- inside the
                   graph with RCCL; with gloo launched between G_comp[p] and G_adam[p])

    are captured, and replay k runs (p = k % S; set r = (k + S - 1) % S receives view k + S - 1,
    S - 1 views ahead; its last reader was step k - 1):

        stream A:  wait geo[p] -> G_comp[p] -> record step[p]
        stream B:  G_geo[r] -> record geo[r]

    (LSR_PG_MERGE=0 or LSR_PG_GEO=fwd: the composite and the step as two graphs, with the event
    comp[p] between them; the geometry then may wait for it.)

    so a replay is one full language step (the loss it returns is that of the view it composited and
    updated from) and later views' geometry overlaps it.  Two graphs on two streams are separate
    queues: unlike one graph with two branches (which this HIP runtime launches on one queue in
    capture order), they run concurrently.  The geometry reads nothing the step
    writes (the language step freezes the geometry, scene/gaussian_model.py:203-217); the step's
    feature fill reads what the previous step's Adam wrote (stream A order).

    A sequence of views (train.py:85-87): pass slots=[ViewSlot(...) for each set] and a
    forward_fn(slot) that renders from the slot; capture(views=[v0, ..., v_{S-2}]) takes the first
    S - 1 views and replay(next_view=v) the view S - 1 replays ahead (it is copied into that view's
    set on the caller's stream, after that set's last reader finished; each set keeps its own camera
    and target, so a replay never pairs one view's geometry with another's target).  Without slots
    forward_fn() renders one fixed view.

    The rasterizer runs in capacity mode (capacities from eager warm-up views, with headroom).  A
    view over capacity is flagged per set and the captured Adam skips on that flag (no parameter,
    moment or step count changes: the view is left out, include/lsr.h lsr_adam_multi); check()
    counts the skipped steps and re-captures.  N > 1: the flag is all-reduced in the same collective
    as the gradients (GradBucket.all_reduce(flag=)), so when one rank's view overflowed EVERY rank
    skips that step and re-captures: the ranks stay identical and no zero gradient is averaged in.
    The collective runs between the backward and Adam graphs (gloo; RCCL at N > 1 by default), or
    inside the step graph when captured (distributed.collective_capturable); the update then also
    fills the next set's records (lsr_adam_fill_language), as the fused tail does at N = 1.

        g = PipelinedGraphStep(lambda: render(...)["language_l1"], [gaussians._language_feature], optimizer)
        for it in range(iterations):
            loss = g.replay()   # this replay's view's loss (on the caller's stream after the replay)
        g.check(); g.sync()

    forward_fn() runs render() + the loss and returns the loss (no backward).  The graphs own the
    parameters' .grad tensors.  Work the caller enqueues on its stream between replays (a .clone()
    of the returned loss) precedes the device work of the replay S - 1 later, not of the next one;
    after changing the parameters or the optimizer state between replays, call follow_caller().

    Rotation mode (rotation=R > 1, N = 1; LSR_PG_ROT): 2 R buffer sets in two groups; every R-th
    replay launches the next R steps as ONE stream-A graph (fewer graph boundaries: ~20-28 us of idle
    queue each at C3) and the following R views' geometry on stream B; the replays in between launch
    nothing.  Parameters, learning rates and check() apply at rotation boundaries (k % R == 0).

    Knobs (measured at C3): LSR_PG_SETS (2 or 3), LSR_PG_GEO=fwd (the geometry starts
    only after this view's compositing), LSR_PG_PRIO=geo|step (stream priorities), LSR_PG_ROT."""

    def __init__(self, forward_fn, params, optimizer, headroom: float = 1.125, warmup: int = 2, bucket=None,
                 slots=None, sets: int = None, rotation: int = None, model=None, bucket_factory=None,
                 ahead: int = None):
        self.forward_fn = forward_fn
        # replay() waits on the host until step k - ahead has finished before enqueuing step k
        # (0: no limit; LSR_PG_AHEAD)
        self.ahead = int(ahead if ahead is not None else os.environ.get("LSR_PG_AHEAD", "0"))
        self.model = model  # its active_sh_degree is part of the capture key (graph.capture_key)
        self.params = [p for p in params]
        self.optimizer = optimizer
        self.bucket = bucket
        self.bucket_factory = bucket_factory  # rebuilds the bucket at a re-capture over replaced parameters
        self.headroom = float(headroom)
        self.warmup = int(warmup)
        dev = self.params[0].device
        # three sets by default: measured at C3 (tools/pg_sweep.py, one box) 0.435 ms per step against
        # 0.482 with two; a view's geometry then runs two steps ahead, beside the backward and the
        # next compositing, and no compositing waits on a cross-stream event that is not yet signalled
        # rotation R > 1: R consecutive steps per stream-A graph over 2 R buffer sets (N = 1 only)
        R = int(rotation if rotation is not None else os.environ.get("LSR_PG_ROT", "1"))
        if R < 1 or (R > 1 and bucket is not None):
            raise ValueError("PipelinedGraphStep: rotation >= 1, and > 1 only without a bucket (N = 1)")
        self.R = R
        S = int(sets if sets is not None else (len(slots) if slots else
                                               (2 * R if R > 1 else os.environ.get("LSR_PG_SETS", "3"))))
        if S < 2:
            raise ValueError("PipelinedGraphStep: at least two buffer sets")
        if R > 1 and S != 2 * R:
            raise ValueError("PipelinedGraphStep: a rotation of R steps takes 2 R buffer sets")
        if slots is not None and len(slots) != S:
            raise ValueError("PipelinedGraphStep: one ViewSlot per buffer set")
        self.S = S
        self.slots = list(slots) if slots is not None else None
        self.sets = tuple(_native.static_buffers() for _ in range(S))
        # A: step, B: geometry.  (Stream priorities measured worse: a high-priority geometry stream
        # 0.82 ms per step, a high-priority step stream 0.57, none 0.48; LSR_PG_PRIO=geo / step)
        prio = os.environ.get("LSR_PG_PRIO", "none")
        # the later view's geometry starts with the step ("start") or after this view's compositing
        # ("fwd": beside the backward and Adam only); measured C3 with 2 sets: start 0.49, fwd 0.54 ms
        self.geo_after_fwd = os.environ.get("LSR_PG_GEO", "start") == "fwd"
        self.streams = (torch.cuda.Stream(dev, priority=-1 if prio == "step" else 0),
                        torch.cuda.Stream(dev, priority=-1 if prio == "geo" else 0))
        self.overflow = tuple(torch.zeros((), dtype=torch.int32, device=dev) for _ in range(S))
        self._one = torch.ones((), device=dev)
        self._reset_graphs()
        self.captures = 0
        self.rendered = self.entries = 0
        self._skipped_base = 0
        self.fused = self.fill_after = self.defer = False  # the update's record fill (set by capture)
        self._tails = [None] * self.S
        self._loaded = [None] * S  # the view each set's slot holds (slots only)
        self._assigned = [None] * S  # rotation mode: the view each set's next geometry renders

    def _reset_graphs(self):
        S = self.S
        self.g_geo, self.g_comp, self.g_step, self.g_adam = [None] * S, [None] * S, [None] * S, [None] * S
        self.grads = [None] * S
        self.static_loss = [None] * S
        self.ev_geo = self.ev_comp = self.ev_step = [None] * S
        self.g_rot = self.g_rot0 = None
        self.k = 0
        self.primed = False

    def _fwd(self, p):
        return self.forward_fn(self.slots[p]) if self.slots is not None else self.forward_fn()

    def _measure(self, min_rendered, min_entries):
        _native.LAST_COUNTS.clear()
        side = torch.cuda.Stream(device=self.params[0].device)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for i in range(self.warmup):
                for p in self.params:
                    p.grad = None
                # every set's view when they differ: the capacities cover the views loaded so far
                self._fwd(i % (self.S - 1)).backward()
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

    def capture(self, min_rendered: int = 0, min_entries: int = 0, views=None):
        """views: the first S - 1 views (camera, gt, mask) when the step renders from ViewSlots (a
        shorter list repeats its last view); the capacities are measured on them."""
        S = self.S
        if self.slots is not None:
            if not views:
                raise ValueError("PipelinedGraphStep.capture: the first views are needed with slots")
            views = list(views)[:S - 1]
            views += [views[-1]] * (S - 1 - len(views))
            for j in range(S - 1):
                self.slots[j].load(*_as_view(views[j]))
                self._loaded[j] = self._assigned[j] = views[j]
        # the optimizer's current tensors (a parameter replaced since the last capture: the capture key
        # changed, replay() re-captures here) and a gradient bucket built over them
        self.params = current_params(self.optimizer, self.params)
        self.bucket = resolve_bucket(self.bucket, self.bucket_factory, self.params)
        # the caller's still-alive autograd graphs keep the parameters' AccumulateGrad nodes bound to
        # their streams: released, so the warm-up and the captures create their own (graph.py)
        self.key = capture_key(self.model, self.optimizer, self.params)
        self.stale_released = release_stale_accumulators(self.params)
        self._measure(min_rendered, min_entries)
        self._reset_graphs()
        self.optimizer.prepare_capture()
        self._skipped_base = self.optimizer.skipped_steps()
        cur = torch.cuda.current_stream()
        sa, sb = self.streams
        for s in self.streams:
            s.wait_stream(cur)
        caps = [_native.capacity(self.rendered, self.entries, self.overflow[p]) for p in range(S)]
        # eager forwards allocate every set at its capacity sizes (no allocation may happen during a
        # capture); nothing is updated
        for p in range(S):
            with torch.cuda.stream(sa), caps[p], self.sets[p]:
                self._fwd(p)
        sb.wait_stream(sa)
        # N > 1: the all-reduce of the gradients (and, in the same collective, of the set's overflow
        # flag: every rank then skips when one view overflowed) inside the step graph when the collective
        # is captured (distributed.collective_capturable: RCCL with one rank, or LSR_GRAPH_COLLECTIVE=1),
        # else launched between the backward and Adam graphs (gloo, and RCCL at N > 1 by default)
        dev = self.params[0].device
        coll_in_graph = self.bucket is not None and collective_capturable()
        self.coll_in_graph = coll_in_graph
        if coll_in_graph:  # the communicator exists before the capture (its creation is not capturable)
            with torch.cuda.stream(sa):
                self.bucket.all_reduce(average=True, flag=torch.zeros((), dtype=torch.int32, device=dev))
            for q in self.params:
                q.grad = None
        # N = 1 language step: Adam inside the backward's epilogue pass, which also writes the updated
        # feature into the NEXT set's records (the next composite needs no fill; the geometry call never
        # writes those slots, so it may run before, during or after)
        fused = self.bucket is None and len(self.params) == 1 and _fused_tail_enabled()
        self.fused = fused
        # N > 1 language step: the update after the all-reduce writes the feature into the next set's
        # records (lsr_adam_fill_language), so every composite but the first after a capture (refilled
        # from the parameter by replay(), _refill) needs no fill either
        fill_after = self.bucket is not None and len(self.params) == 1 and _fused_tail_enabled()
        self.fill_after = fill_after
        # ... and the gradient epilogue moves behind the collective: the backward leaves the language
        # partials (include/lsr.h LSR_BWD_DEFER_TAIL), the all-reduce averages them, and ONE pass
        # (lsr_language_tail) writes the gradients, steps and fills -- the N = 1 tail with the collective
        # before it (LSR_PG_DEFER=0: the epilogue in the backward, the collective over .grad, then
        # lsr_adam_fill_language)
        defer = fill_after and self.bucket.direct and os.environ.get("LSR_PG_DEFER", "1") != "0"
        self.defer = defer
        self._tails = [None] * S
        comp_phase = (_native.forward_phase.COMPOSITE_FILLED if fused or fill_after
                      else _native.forward_phase.COMPOSITE)
        # fused: the first composite after a capture fills set 0's feature records itself (G_comp0, run
        # by replay k = 0 instead of G_comp[0]; it owns its own gradients, grads0); later sets are
        # filled by the step before
        self.g_comp0 = None
        self.grads0 = None
        # the composite and the step in ONE graph per set (default): a graph boundary on stream A
        # costs ~16-24 us of idle queue at C3 (rocprofv3 trace, round 4), and nothing needs the point
        # between them unless the geometry waits for the compositing (LSR_PG_GEO=fwd)
        merged = not self.geo_after_fwd and os.environ.get("LSR_PG_MERGE", "1") != "0"
        self.merged = merged

        def update_ctx(p):
            if defer:  # this set's deferred tail (its arguments stay with the context)
                self._tails[p] = _native.fused_update(self.optimizer, self.params[0], skip=self.overflow[p],
                                                      fill=self._record_ptr((p + 1) % S), defer=True)
                return self._tails[p]
            return _native.fused_update(self.optimizer, self.params[0], skip=self.overflow[p],
                                        fill=self._record_ptr((p + 1) % S)) if fused else _nullctx()

        def adam_fill(p):  # (N > 1) the set's update fills the next set's records
            return (self._record_ptr((p + 1) % S), _native.RAW_LANGUAGE) if fill_after else None

        def step_body(p, loss):
            with update_ctx(p):  # the backward runs on its forward's stream (sa)
                loss.backward(self._one)  # dL/dloss = 1 from a static tensor: no seed-fill kernel
                if coll_in_graph:
                    self._collective(p)
                if defer:
                    if coll_in_graph:
                        self._tails[p].run_tail()
                elif self.bucket is None or coll_in_graph:
                    self.optimizer.step(skip=self.overflow[p], fill=adam_fill(p))

        geo_delay = int(os.environ.get("LSR_PG_GEO_DELAY_US", "0"))
        step_delay = int(os.environ.get("LSR_PG_STEP_DELAY_US", "0"))
        for p in range(S):
            if self.R > 1:
                continue  # geometry and steps are captured per rotation group below
            g = torch.cuda.CUDAGraph()
            with graph_capture(g, stream=sb), caps[p], self.sets[p], \
                    _native.forward_phase(_native.forward_phase.GEOMETRY):
                if geo_delay:  # measurement knob: the geometry stream starts later in each step
                    _native._check(_native.load().lsr_debug_delay(geo_delay, _native._stream(dev)), "delay")
                self._fwd(p)  # its outputs are written by the composite half
            self.g_geo[p] = g
            for q in self.params:
                q.grad = None  # the captured backward assigns its own .grad (no accumulate)
            if fused and p == 0:
                g = torch.cuda.CUDAGraph()
                with graph_capture(g, stream=sa):
                    with caps[p], self.sets[p], _native.forward_phase(_native.forward_phase.COMPOSITE):
                        loss = self._fwd(p)
                    if merged:
                        step_body(p, loss)
                if merged:
                    self.grads0 = [q.grad for q in self.params]
                    del loss
                    for q in self.params:
                        q.grad = None
                else:
                    del loss
                self.g_comp0 = g
            g = torch.cuda.CUDAGraph()
            with graph_capture(g, stream=sa):
                if step_delay:  # measurement knob: the step stream starts each step later
                    _native._check(_native.load().lsr_debug_delay(step_delay, _native._stream(dev)), "delay")
                with caps[p], self.sets[p], _native.forward_phase(comp_phase):
                    loss = self._fwd(p)
                if merged:
                    step_body(p, loss)
            self.g_comp[p] = g
            if not merged:
                g = torch.cuda.CUDAGraph()
                with graph_capture(g, stream=sa):
                    step_body(p, loss)
                self.g_step[p] = g
            self.grads[p] = [q.grad for q in self.params]  # this set's graph-owned gradients
            if self.bucket is not None and not coll_in_graph:  # the all-reduce sits between two graphs
                g = torch.cuda.CUDAGraph()
                with graph_capture(g, stream=sa):
                    if defer:
                        self._tails[p].run_tail()
                    else:
                        self.optimizer.step(skip=self.overflow[p], fill=adam_fill(p))
                self.g_adam[p] = g
            self.static_loss[p] = loss.detach()  # the set's static loss tensor
            del loss
        if self.R > 1:
            self._capture_rotations(caps, comp_phase, fused, step_body)
        cur.wait_stream(sa)
        cur.wait_stream(sb)
        self.ev_rot = [torch.cuda.Event() for _ in range(2)]
        self.ev_geo = [torch.cuda.Event() for _ in range(S)]
        self.ev_comp = [torch.cuda.Event() for _ in range(S)]
        self.ev_step = [torch.cuda.Event() for _ in range(S)]
        self.ev_cur = [torch.cuda.Event() for _ in range(S)]
        self._since_capture = 0
        self._fast = False
        self._launchers = {}  # (set, fast) -> _native.GraphLauncher (replay's steady state)
        self._refill = fill_after  # the first composite's records: from the parameter (replay)
        self.captures += 1
        return self

    def _capture_rotations(self, caps, comp_phase, fused, step_body):
        """Rotation mode: per group j of R sets (j = 0: sets 0..R-1, j = 1: sets R..2R-1) one graph
        of R full steps, composite + loss + backward + Adam each (and, fused, a variant of group 0
        whose first composite fills its own records, for the first replay after a capture)."""
        R, sa = self.R, self.streams[0]

        def rot(j, first):
            g = torch.cuda.CUDAGraph()
            grads = []
            with graph_capture(g, stream=sa):
                for p in range(j * R, (j + 1) * R):
                    for q in self.params:
                        q.grad = None  # each step's backward assigns its own .grad
                    phase = _native.forward_phase.COMPOSITE if (first and p == 0) else comp_phase
                    with caps[p], self.sets[p], _native.forward_phase(phase):
                        loss = self._fwd(p)
                    step_body(p, loss)
                    grads.append([q.grad for q in self.params])
                    self.static_loss[p] = loss.detach()  # the set's static loss (same tensor in every graph)
                    del loss
            return g, grads

        self.g_rot = [rot(0, False), rot(1, False)]
        self.g_rot0 = rot(0, True) if fused else None
        # each group's R geometries as one stream-B graph as well
        sb = self.streams[1]
        self.g_geo_rot = []
        for j in range(2):
            g = torch.cuda.CUDAGraph()
            with graph_capture(g, stream=sb):
                for p in range(j * R, (j + 1) * R):
                    with caps[p], self.sets[p], _native.forward_phase(_native.forward_phase.GEOMETRY):
                        self._fwd(p)
            self.g_geo_rot.append(g)
        for j in range(2):
            for i, gr in enumerate(self.g_rot[j][1]):
                self.grads[j * R + i] = gr

    def _replay_rotation(self, next_view, wait):
        """replay() in rotation mode: at a rotation start (k % R == 0) the group's R steps are launched
        as one graph on stream A, and the next rotation's geometry (the other group, whose sets the
        previous rotation released) on stream B; the other replays launch nothing."""
        S, R = self.S, self.R
        sa, sb = self.streams
        cur = torch.cuda.current_stream()
        k = self.k
        if next_view is not None:
            if self.slots is None:
                raise RuntimeError("PipelinedGraphStep.replay(next_view=...) needs ViewSlots")
            self._assigned[(k + S - 1) % S] = next_view
        if k % R == 0:
            j = (k // R) % 2
            if not self.primed:  # group 0's geometry (its views were loaded at capture)
                sb.wait_stream(cur)
                with torch.cuda.stream(sb):
                    self.g_geo_rot[0].replay()
                self.ev_geo[0].record(sb)
                self.primed = True
            if wait or self._since_capture == 0:
                sa.wait_stream(cur)  # the caller's earlier work (parameters, learning rates) first
            sa.wait_event(self.ev_geo[j * R])  # the group's geometry graph
            with torch.cuda.stream(sa):
                self.optimizer.sync_lr()
                if self._refill and self.fused and not (k == 0 and self.g_rot0 is not None):
                    self._refill_records(j * R)  # the caller changed the parameter (follow_caller)
                self._refill = False
                g, _ = self.g_rot0 if (k == 0 and self.g_rot0 is not None) else self.g_rot[j]
                g.replay()
            self.ev_rot[j].record(sa)
            # the other group's sets were last read by the previous rotation (none before the first)
            o = 1 - j
            if k >= R:
                sb.wait_event(self.ev_rot[o])
            if self.slots is not None:
                sb.wait_stream(cur)  # the views' tensors
            for p in range(o * R, (o + 1) * R):
                if self.slots is not None and self._assigned[p] is not None:
                    view = _as_view(self._assigned[p])
                    with torch.cuda.stream(sb):
                        self.slots[p].load(*view)
                    for t in self.slots[p].sources(*view):
                        t.record_stream(sb)
                    self._loaded[p] = self._assigned[p]
            with torch.cuda.stream(sb):
                self.g_geo_rot[o].replay()
            self.ev_geo[o * R].record(sb)
            if wait:
                cur.wait_event(self.ev_rot[j])
        elif wait:
            cur.wait_event(self.ev_rot[(k // R) % 2])
        self._since_capture += 1
        self.k += 1
        return self.static_loss[k % S]

    def _collective(self, p):
        """Set p's step collective (N > 1): the deferred backward's language partials, or the .grad
        tensors, with the set's overflow flag."""
        if self.defer:  # the partials carry the set's overflow flag themselves (include/lsr.h)
            self.bucket.all_reduce_partials(self._tails[p].partials(), average=True)
        else:
            self.bucket.all_reduce(average=True, flag=self.overflow[p])

    def _record_ptr(self, p):
        """Device address of set p's per-Gaussian render records (include/lsr.h lsr_state_layout.record)."""
        geom = self.sets[p].tensors[("scratch", _native.LSR_BUF_GEOM)]
        _, H, W = self.sets[p].tensors[("out", "color")].shape
        P = int(self.params[0].shape[0])
        return geom.data_ptr() + _native.state_layout(P, int(W), int(H), 0)["record"]

    def _geometry(self, r, after=None, released=None):
        """Set r's geometry graph on stream B, after everything the caller's stream holds (the set's
        view loaded, its last reader finished) or, with `released` (an event: the set's last reader
        done), after that alone [and after `after`]."""
        sb = self.streams[1]
        if released is not None:
            sb.wait_event(released)
        else:
            sb.wait_stream(torch.cuda.current_stream())
        if after is not None:
            sb.wait_event(after)
        with torch.cuda.stream(sb):
            self.g_geo[r].replay()
        self.ev_geo[r].record(sb)

    def _launcher(self, p, fast):
        """Set p's steady-state stream-A launch (replay): after the caller's mark of replay k - S + 1
        (ev_cur[p + 1], not in the fast form) and set p's geometry, the step graph, then ev_step[p].
        None until every one of those events exists (torch creates an event at its first record)."""
        if not _NATIVE_LAUNCH:
            return None
        key = (p, fast)
        fn = self._launchers.get(key)
        if fn is None:
            S = self.S
            waits = ([] if fast else [self.ev_cur[(p + 1) % S]]) + [self.ev_geo[p]]
            if any(e.cuda_event == 0 for e in waits + [self.ev_step[p]]):
                return None
            fn = _native.GraphLauncher(self.g_comp[p], self.streams[0], waits, self.ev_step[p])
            self._launchers[key] = fn
        return fn

    def replay(self, next_view=None, wait: bool = True) -> torch.Tensor:
        """One language step of the view loaded S - 1 replays ago (or at capture); next_view
        (camera, gt, mask) is the view of the replay S - 1 ahead (ViewSlots only; None: the view of
        its set stays).

        wait=False: the caller's stream is not chained to the replay -- the returned loss (and the
        graph-owned gradients) are valid on it only after synchronize() (and only those of the
        last S replays: a set's next composite rewrites them), and nothing of the replay
        goes through the caller's stream (its queue carries no event or wait per step: on this
        runtime the two streams' packets can share a hardware queue with it, and a wait there held
        stream A ~20-28 us per step).  The caller must not change the parameters
        between such replays without follow_caller().  bench.py times this form, with the
        synchronize() inside the timed region."""
        if self.g_comp[0] is None and getattr(self, "g_rot", None) is None:
            self.capture()
        elif (self.R == 1 or self.k % self.R == 0) and capture_key(self.model, self.optimizer, self.params) != self.key:
            # an SH-degree step or replaced parameters since the capture
            self._recapture(self.rendered, self.entries)
        if self.R > 1:
            return self._replay_rotation(next_view, wait)
        S = self.S
        sa, sb = self.streams
        p = self.k % S
        r = (self.k + S - 1) % S
        if 0 < self.ahead < S and self._since_capture >= self.ahead:
            # host throttle: at most `ahead` steps enqueued beyond the running one (the queues stay
            # short; a step's stream-A work still follows the previous step without a host gap)
            self.ev_step[(self.k - self.ahead) % S].synchronize()
        fast = not wait and self._since_capture >= S - 1
        if wait and self._fast:  # back from fast replays: the lagged events were not recorded
            self._since_capture = 0
        # the caller's stream object (~2.4 us of host time) only where it is used before the launch
        cur = torch.cuda.current_stream() if (next_view is not None or not self.primed
                                               or self._since_capture < S - 1) else None
        if not self.primed:  # the first S - 1 views' geometry (nothing ran since the capture)
            for j in range(S - 1):
                self._geometry((self.k + j) % S)
            self.primed = True
        self._fast = fast
        # set r's last reader was step k - 1 (the view S - 1 ahead goes there)
        released = self.ev_step[(self.k - 1) % S] if self.k > 0 else None
        if next_view is not None:
            if self.slots is None:
                raise RuntimeError("PipelinedGraphStep.replay(next_view=...) needs ViewSlots")
            if fast:
                # on stream B, after step k - 1 and after the caller's stream (the view's tensors)
                sb.wait_stream(cur)
                if released is not None:
                    sb.wait_event(released)
                view = _as_view(next_view)
                with torch.cuda.stream(sb):
                    self.slots[r].load(*view)
                for t in self.slots[r].sources(*view):
                    t.record_stream(sb)
            else:
                # the caller's stream waited for step k - 1 at the end of the previous replay
                self.slots[r].load(*_as_view(next_view))
            self._loaded[r] = next_view
        first = self.k == 0 and self.g_comp0 is not None
        refill = self._refill and (self.fused or self.fill_after) and not first
        # Steady state (the merged step graph, no update graph, no refill): the stream-A waits, the
        # launch and the step's event in ONE native call (lsr_graph_launch); the Python path below
        # costs ~8 us more host time before the launch, which a loss.item() loop pays every step
        launcher = (self._launcher(p, fast) if self.merged and self.g_adam[p] is None and not first and not refill
                    and self._since_capture >= S - 1 else None)
        if launcher is not None:
            self._since_capture += 1
            self.optimizer.sync_lr(stream=sa)
            self._refill = False
            launcher()
        else:
            if not fast:
                # Stream A does not wait for the caller's stream as it is now: that stream waits for the
                # previous step (below), so the wait would be a round trip between two queues (measured
                # ~35 us of idle stream A per step at C3).  It waits instead for the
                # caller's work up to the start of replay k - S + 1, long done: the caller's uses of the
                # loss of replay k - S (whose tensor composite k rewrites) precede that.  The first
                # S - 1 replays after a capture wait for the caller's stream itself.  (This replay's own
                # mark on the caller's stream, ev_cur[k], is recorded after the step's launch below: the
                # caller's stream gets nothing from replay() before it, and a synced loop's stream A
                # idles until the launch.)
                if self._since_capture < S - 1:
                    sa.wait_stream(cur)
                else:
                    sa.wait_event(self.ev_cur[(self.k + 1) % S])  # recorded at replay k - S + 1
            self._since_capture += 1
            sa.wait_event(self.ev_geo[p])
            with torch.cuda.stream(sa):
                self.optimizer.sync_lr()  # a changed learning rate: a host-to-device copy on stream A
                if refill:
                    # the caller changed the parameter (follow_caller), or the first composite after an
                    # N > 1 capture (its records were filled by no earlier update)
                    self._refill_records(p)
                self._refill = False
                (self.g_comp0 if first else self.g_comp[p]).replay()
                if not self.merged:
                    self.ev_comp[p].record(sa)
                    self.g_step[p].replay()
                if self.g_adam[p] is not None:
                    for q, g in zip(self.params, self.grads[p]):
                        q.grad = g
                    self._collective(p)
                    self.g_adam[p].replay()
            self.ev_step[p].record(sa)
        if cur is None:
            cur = torch.cuda.current_stream()
        if not fast:
            self.ev_cur[self.k % S].record(cur)
        # view k + S - 1's geometry into set r
        after = self.ev_comp[p] if self.geo_after_fwd and not self.merged else None
        if fast:
            # the set's view (if any) was loaded on stream B itself
            self._geometry(r, after=after, released=self.ev_step[(self.k - 1) % S])
        else:
            self._geometry(r, after=after)
            cur.wait_event(self.ev_step[p])
        self.k += 1
        return self.static_loss[p]

    def last_grads(self):
        """The gradient tensors the last replay wrote (graph-owned; the first replay after a fused
        capture has its own)."""
        if self.k == 0:
            raise RuntimeError("PipelinedGraphStep.last_grads: no replay yet")
        if self.R > 1 and self.k <= self.R and self.g_rot0 is not None:
            return self.g_rot0[1][self.k - 1]
        if self.k == 1 and self.merged and self.g_comp0 is not None:
            return self.grads0
        return self.grads[(self.k - 1) % self.S]

    def follow_caller(self):
        """The next replays wait for everything the caller's stream holds now (e.g. parameters the
        caller changed between replays).  With the fused tail the previous step already wrote the
        updated feature into the next set's records (COMPOSITE_FILLED never re-reads the parameter):
        the next replay refills them from the parameter first."""
        self._since_capture = 0
        self._refill = True

    def _refill_records(self, p):
        """Set p's records' language slots from the parameter as it is now (on the current stream),
        for a composite that would otherwise blend what the previous step's fused tail wrote."""
        radii = self.sets[p].tensors[("out", "radii")]
        _native.fill_language(self.params[0], _native.RAW_LANGUAGE, radii, self._record_ptr(p))

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
        capacities and return False: the over-capacity views were not rasterized, and at N = 1 their
        steps changed nothing (optimizer.skipped_steps() counts them; train those views again).
        Rotation mode: only between rotations (k % R == 0), where no launched step is pending."""
        if self.R > 1 and self.k % self.R != 0:
            raise RuntimeError("PipelinedGraphStep.check: in rotation mode only at a rotation boundary")
        self.synchronize()
        skipped = self.optimizer.skipped_steps() - self._skipped_base
        if skipped == 0 and all(int(o.item()) == 0 for o in self.overflow):
            return True
        for o in self.overflow:
            o.zero_()
        self._recapture(2 * self.rendered, 2 * self.entries)
        return False

    def _recapture(self, min_rendered, min_entries):
        """Capture again, continuing with the views already loaded for the next S - 1 steps."""
        self.synchronize()
        self.sync()
        src = self._assigned if self.R > 1 else self._loaded
        views = [src[(self.k + j) % self.S] for j in range(self.S - 1)] if self.slots else None
        self.capture(min_rendered, min_entries, views=views)
