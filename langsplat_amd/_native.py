"""ctypes binding of liblsr.so (the C ABI in include/lsr.h).

This is the reference-side binding a maintainer would add in place of the CUDA extension's
pybind module `diff_gaussian_rasterization._C`.  Tensors are passed as raw
device pointers; scratch buffers are torch uint8 tensors handed out through the allocator
callback (so the caching allocator owns them and autograd keeps them alive for backward).

There is no CPU fallback: if liblsr.so cannot be loaded the import of this module fails.
"""
from __future__ import annotations

import ctypes
import math
import os
import threading
from typing import Dict, Optional

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# LSR_LIB: a measurement variant built by tools/build_variant.py (same-box A/B); default the product
LIB_PATH = os.environ.get("LSR_LIB") or os.path.join(_HERE, "liblsr.so")

LSR_BUF_GEOM, LSR_BUF_BINNING, LSR_BUF_IMAGE, LSR_BUF_BACKWARD = 0, 1, 2, 3
ABI_VERSION = 17
ADAM_STEP_WORDS = 66  # include/lsr.h LSR_ADAM_STEP_WORDS
ADAM_WORD_SKIPPED, ADAM_WORD_LR = 49, 50  # LSR_ADAM_WORD_SKIPPED / LSR_ADAM_WORD_LR
# lsr_raw_flags (include/lsr.h): inputs are GaussianModel's raw parameters
RAW_OPACITY, RAW_SCALES, RAW_ROTATIONS, RAW_LANGUAGE = 1, 2, 4, 8
FWD_ZERO_GRAD_RECORDS, FWD_NO_COLOR_GRAD, FWD_NO_BACKWARD = 1, 2, 4  # lsr_forward_flags
BWD_RECORDS_ZEROED, BWD_SHARED_CU, BWD_DEFER_TAIL = 1, 2, 4  # lsr_backward_flags
_vp = ctypes.c_void_p


class LsrSettings(ctypes.Structure):
    _fields_ = [
        ("image_height", ctypes.c_int32),
        ("image_width", ctypes.c_int32),
        ("tanfovx", ctypes.c_float),
        ("tanfovy", ctypes.c_float),
        ("scale_modifier", ctypes.c_float),
        ("sh_degree", ctypes.c_int32),
        ("prefiltered", ctypes.c_int32),
        ("debug", ctypes.c_int32),
        ("include_feature", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("bg", _vp),
        ("viewmatrix", _vp),
        ("projmatrix", _vp),
        ("campos", _vp),
    ]


class LsrForwardArgs(ctypes.Structure):
    _fields_ = [("P", ctypes.c_int32), ("M", ctypes.c_int32)] + [
        (n, _vp) for n in ("means3D", "shs", "colors_precomp", "language_feature", "opacities", "scales",
                           "rotations", "cov3D_precomp", "out_color", "out_language_feature", "radii")
    ] + [("raw", ctypes.c_int32), ("flags", ctypes.c_int32), ("shs_rest", _vp), ("visible", _vp),
         ("loss_target", _vp), ("loss_mask", _vp), ("out_loss", _vp), ("capacity_rendered", ctypes.c_int64),
         ("capacity_entries", ctypes.c_int64), ("overflow", _vp), ("out_num_entries", ctypes.POINTER(ctypes.c_int64)),
         ("language_ready", _vp), ("phase", ctypes.c_int32)]


class LsrAdamTensor(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("param", _vp), ("grad", _vp), ("exp_avg", _vp), ("exp_avg_sq", _vp),
                ("lr", ctypes.c_double), ("beta1", ctypes.c_double), ("beta2", ctypes.c_double),
                ("eps", ctypes.c_double), ("step", ctypes.c_int64)]


class LsrBackwardArgs(ctypes.Structure):
    _fields_ = [("P", ctypes.c_int32), ("M", ctypes.c_int32), ("num_rendered", ctypes.c_int64)] + [
        (n, _vp) for n in ("means3D", "shs", "colors_precomp", "language_feature", "opacities", "scales",
                           "rotations", "cov3D_precomp", "radii", "dL_dout_color", "dL_dout_language_feature",
                           "geom_buffer", "binning_buffer", "image_buffer", "dL_dmeans2D", "dL_dcolors",
                           "dL_dlanguage_feature", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh",
                           "dL_dscales", "dL_drotations")
    ] + [("raw", ctypes.c_int32), ("flags", ctypes.c_int32), ("shs_rest", _vp), ("dL_dsh_rest", _vp),
         ("dL_dloss", _vp), ("update", ctypes.POINTER(LsrAdamTensor)), ("update_step_dev", _vp),
         ("update_skip", _vp), ("fill_record", _vp)]


class LsrStateLayout(ctypes.Structure):
    _fields_ = [(n, ctypes.c_size_t) for n in (
        "depth_key", "tiles_touched", "rect", "record", "clamped", "sorted_ids", "super_offset",
        "counters", "ranges", "final_T", "n_contrib", "point_list", "grad_records")]


class LsrKernelStat(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 32), ("launches", ctypes.c_int64), ("total_ms", ctypes.c_double)]


ALLOC_FN = ctypes.CFUNCTYPE(_vp, _vp, ctypes.c_int32, ctypes.c_size_t)

# symbol -> (restype, argtypes); must cover every function declared in include/lsr.h
SIGNATURES = {
    "lsr_abi_version": (ctypes.c_int32, []),
    "lsr_last_error": (ctypes.c_char_p, []),
    "lsr_geom_bytes": (ctypes.c_size_t, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    "lsr_image_bytes": (ctypes.c_size_t, [ctypes.c_int32, ctypes.c_int32]),
    "lsr_binning_bytes": (ctypes.c_size_t, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int64]),
    "lsr_backward_bytes": (ctypes.c_size_t, [ctypes.c_int32]),
    "lsr_state_layout_of": (ctypes.c_int32, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64,
                                             ctypes.POINTER(LsrStateLayout)]),
    "lsr_forward": (ctypes.c_int32, [ctypes.POINTER(LsrSettings), ctypes.POINTER(LsrForwardArgs), ALLOC_FN, _vp,
                                     _vp, ctypes.POINTER(ctypes.c_int64)]),
    "lsr_backward": (ctypes.c_int32, [ctypes.POINTER(LsrSettings), ctypes.POINTER(LsrBackwardArgs), ALLOC_FN, _vp,
                                      _vp]),
    "lsr_mark_visible": (ctypes.c_int32, [ctypes.c_int32, _vp, _vp, _vp, _vp, _vp]),
    "lsr_fill_language": (ctypes.c_int32, [ctypes.c_int32, _vp, ctypes.c_int32, _vp, _vp, _vp]),
    "lsr_adam_step": (ctypes.c_int32, [ctypes.c_int64, _vp, _vp, _vp, _vp, ctypes.c_double, ctypes.c_double,
                                       ctypes.c_double, ctypes.c_double, ctypes.c_int64, _vp]),
    "lsr_adam_multi": (ctypes.c_int32, [ctypes.c_int32, ctypes.POINTER(LsrAdamTensor), ctypes.c_float, _vp, _vp,
                                        _vp]),
    "lsr_adam_fill_language": (ctypes.c_int32, [ctypes.POINTER(LsrAdamTensor), ctypes.c_float, _vp, _vp, _vp,
                                                ctypes.c_int32, _vp]),
    "lsr_language_tail": (ctypes.c_int32, [ctypes.POINTER(LsrSettings), ctypes.POINTER(LsrBackwardArgs), _vp]),
    "lsr_densification_stats": (ctypes.c_int32, [ctypes.c_int32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "lsr_dist_cuda2": (ctypes.c_int32, [ctypes.c_int64, _vp, _vp, ALLOC_FN, _vp, _vp]),
    "lsr_masked_l1_scratch_bytes": (ctypes.c_size_t, [ctypes.c_int32, ctypes.c_int64]),
    "lsr_masked_l1_forward": (ctypes.c_int32, [ctypes.c_int32, ctypes.c_int64, _vp, _vp, _vp, ctypes.c_int32, _vp, _vp,
                                               _vp]),
    "lsr_masked_l1_backward": (ctypes.c_int32, [ctypes.c_int32, ctypes.c_int64, _vp, _vp, _vp, ctypes.c_int32, _vp,
                                                _vp, _vp]),
    "lsr_decode_language_feature": (ctypes.c_int32, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _vp,
                                                     ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _vp, _vp, _vp,
                                                     _vp]),
    "lsr_debug_scan_stalls": (ctypes.c_int32, []),
    "lsr_debug_set_spin_limit": (ctypes.c_uint32, [ctypes.c_uint32]),
    "lsr_debug_bucket_timeline": (ctypes.c_int32, [ctypes.POINTER(ctypes.c_uint32), ctypes.c_int32]),
    "lsr_debug_clock_probe": (ctypes.c_int32, [_vp, _vp]),
    "lsr_debug_delay": (ctypes.c_int32, [ctypes.c_uint32, _vp]),
    "lsr_graph_launch": (ctypes.c_int32, [_vp, _vp, ctypes.POINTER(_vp), ctypes.c_int32, _vp]),
    "lsr_debug_render_stats": (ctypes.c_int32, [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int32]),
    "lsr_debug_render_timeline": (ctypes.c_int32, [ctypes.c_int32, ctypes.POINTER(ctypes.c_uint32), ctypes.c_int32]),
    "lsr_profile_enable": (ctypes.c_int32, [ctypes.c_int32]),
    "lsr_profile_report": (ctypes.c_int32, [ctypes.POINTER(LsrKernelStat), ctypes.c_int32]),
    "lsr_profile_select": (ctypes.c_int32, [ctypes.c_char_p]),
    "lsr_profile_sample": (ctypes.c_int32, [ctypes.c_int32]),
}

_lib: Optional[ctypes.CDLL] = None


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load liblsr.so (building it first if it is absent and hipcc is available)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        from . import build as _build  # compiles the HIP sources; not a fallback path
        _build.build()
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.lsr_abi_version() != ABI_VERSION:
        raise RuntimeError("liblsr.so ABI version mismatch")
    _lib = lib
    return lib


_autograd = None


def autograd_helper():
    """The _lsr_autograd extension (csrc/lsr_autograd.cpp: a leaf tensor's cached AccumulateGrad node,
    read and released; host code), built in-tree first if it is absent."""
    global _autograd
    if _autograd is None:
        if not os.path.exists(os.path.join(_HERE, "_lsr_autograd.so")):
            from . import build as _build
            _build.build_autograd_helper()
        from . import _lsr_autograd
        _autograd = _lsr_autograd
    return _autograd


def last_error() -> str:
    return load().lsr_last_error().decode(errors="replace")


def _check(status: int, what: str):
    if status != 0:
        raise RuntimeError(f"{what} failed (status {status}): {last_error()}")


class GraphLauncher:
    """One captured graph's launch on one stream after given events, with an event recorded after it
    (lsr_graph_launch): the raw handles are read once, so a call costs one ctypes round trip instead
    of torch's stream context, event waits and CUDAGraph.replay() (pipeline.py's synced replays)."""

    def __init__(self, graph: "torch.cuda.CUDAGraph", stream: "torch.cuda.Stream", waits, record):
        self._lib = load()
        self._exec = _vp(graph.raw_cuda_graph_exec())
        if not self._exec.value:
            raise RuntimeError("GraphLauncher: the graph has no instantiated executable")
        self._stream = _vp(stream.cuda_stream)
        self._events = list(waits) + [record]  # kept alive with their handles
        self._waits = (_vp * max(1, len(waits)))(*[e.cuda_event for e in waits])
        self._n = len(waits)
        self._record = _vp(record.cuda_event) if record is not None else None

    def __call__(self):
        _check(self._lib.lsr_graph_launch(self._exec, self._stream, self._waits, self._n, self._record),
               "lsr_graph_launch")


def _ptr(t: Optional[torch.Tensor]):
    if t is None or t.numel() == 0:
        return None
    return ctypes.c_void_p(t.data_ptr())


def _stream(device: torch.device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class _Allocator:
    """Hands out torch uint8 device tensors for the ABI's scratch requests.

    One process-wide ctypes callback (creating a CFUNCTYPE per call costs more than the whole
    binding); the allocator active on this thread is published through a thread-local.
    """

    _tls = threading.local()

    def __init__(self, device: torch.device):
        self.device = device
        self.buffers: Dict[int, torch.Tensor] = {}

    def __enter__(self):
        self._prev = getattr(_Allocator._tls, "active", None)
        _Allocator._tls.active = self
        return self

    def __exit__(self, *exc):
        _Allocator._tls.active = self._prev

    def get(self, which: int) -> torch.Tensor:
        t = self.buffers.get(which)
        return t if t is not None else torch.empty((0,), dtype=torch.uint8, device=self.device)


def _alloc_cb(user, which, nbytes):
    a = getattr(_Allocator._tls, "active", None)
    if a is None:
        return None
    try:
        n = max(int(nbytes), 1)
        st = static_buffers.active()
        t = st.tensor(("scratch", int(which)), (n,), torch.uint8, a.device, at_least=True) if st is not None \
            else torch.empty((n,), dtype=torch.uint8, device=a.device)
    except Exception:  # noqa: BLE001 -- reported to C as NULL -> LSR_ERR_ALLOC
        return None
    a.buffers[int(which)] = t
    return t.data_ptr()


_ALLOC_CB = ALLOC_FN(_alloc_cb)


def _f32c(t: torch.Tensor) -> torch.Tensor:
    if t.dtype != torch.float32:
        t = t.to(torch.float32)
    return t if t.is_contiguous() else t.contiguous()


class _on_device:
    """torch.cuda.device(...) only when it is not already the current device."""

    def __init__(self, device: torch.device):
        idx = device.index if device.index is not None else torch.cuda.current_device()
        self.ctx = None if idx == torch.cuda.current_device() else torch.cuda.device(idx)

    def __enter__(self):
        if self.ctx is not None:
            self.ctx.__enter__()

    def __exit__(self, *exc):
        if self.ctx is not None:
            self.ctx.__exit__(*exc)


class capacity:
    """Within the block, the rasterizer forwards of this thread run in capacity mode (include/lsr.h
    lsr_forward_args.capacity_*): buffers and launch grids sized from `rendered` tile instances and
    `entries` super-tile entries, no wait for the device -- what a HIP graph capture of the step needs
    (langsplat_amd.graph).  `overflow`: a () int32 device tensor each forward sets to 0, or when its
    view exceeds a capacity (it is then not rasterized) to the bits of 1.0f (non-zero as an int; 1.0
    through overflow.view(torch.float32), which GradBucket.all_reduce(flag=) reduces over ranks)."""

    _tls = threading.local()

    def __init__(self, rendered: int, entries: int, overflow: torch.Tensor):
        if rendered <= 0 or entries <= 0:
            raise ValueError("capacity: both capacities must be positive")
        if overflow.dtype != torch.int32 or overflow.numel() != 1:
            raise ValueError("capacity: overflow must be a one-element int32 tensor")
        self.rendered, self.entries, self.overflow = int(rendered), int(entries), overflow

    @staticmethod
    def active():
        return getattr(capacity._tls, "cur", None)

    def __enter__(self):
        self._prev = capacity.active()
        capacity._tls.cur = self
        return self

    def __exit__(self, *exc):
        capacity._tls.cur = self._prev


class language_ready:
    """Within the block, the rasterizer forwards of this thread defer the language feature
    (include/lsr.h lsr_forward_args.language_ready): preprocess, depth order and binning run at
    once, and the stream waits for `event` (a torch.cuda.Event recorded after the language feature's
    last update, on any stream) only before the feature enters the records and the compositing
    starts.  event None: off (the block is a no-op)."""

    _tls = threading.local()

    def __init__(self, event):
        self.event = event

    @staticmethod
    def active():
        return getattr(language_ready._tls, "cur", None)

    def __enter__(self):
        self._prev = language_ready.active()
        language_ready._tls.cur = self.event
        return self

    def __exit__(self, *exc):
        language_ready._tls.cur = self._prev


class forward_phase:
    """Within the block, the rasterizer forwards of this thread enqueue one half of the forward
    (include/lsr.h lsr_forward_args.phase; capacity mode only): GEOMETRY = preprocess, depth order
    and binning; COMPOSITE = the language feature into the records, the compositing and the fused
    loss, into the buffers the geometry call of the same static_buffers set wrote; COMPOSITE_FILLED =
    the same without the feature fill (a fused update wrote the records' language slots: fused_update
    with fill)."""

    GEOMETRY, COMPOSITE, COMPOSITE_FILLED = 1, 2, 3
    _tls = threading.local()

    def __init__(self, phase: int):
        if phase not in (0, 1, 2, 3):
            raise ValueError("forward_phase: 0 (all), 1 (geometry), 2 (composite) or 3 (composite, feature "
                             "already in the records)")
        self.phase = int(phase)

    @staticmethod
    def active() -> int:
        return getattr(forward_phase._tls, "cur", 0)

    def __enter__(self):
        self._prev = forward_phase.active()
        forward_phase._tls.cur = self.phase
        return self

    def __exit__(self, *exc):
        forward_phase._tls.cur = self._prev


class static_buffers:
    """Within the block, the rasterizer forwards of this thread put their scratch buffers and output
    tensors into this object's persistent tensors instead of fresh allocations: the same addresses at
    every forward.  A pipelined graph step (langsplat_amd.pipeline.PipelinedGraphStep) captures a
    backward that reads what a forward captured in ANOTHER graph writes, so both must name the same
    memory.  Tensors are (re)allocated only when a request does not fit (never during a capture)."""

    _tls = threading.local()

    def __init__(self):
        self.tensors: Dict[tuple, torch.Tensor] = {}

    @staticmethod
    def active():
        return getattr(static_buffers._tls, "cur", None)

    def tensor(self, key, shape, dtype, device, at_least=False):
        """The persistent tensor `key` of `shape` (at_least: a 1-D tensor of at least shape[0] elements,
        a view of its first shape[0])."""
        t = self.tensors.get(key)
        fits = t is not None and t.dtype == dtype and t.device == torch.device(device) and (
            t.numel() >= shape[0] if at_least else tuple(t.shape) == tuple(shape))
        if not fits:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError(f"static_buffers: {key} {tuple(shape)} does not fit during a capture")
            t = torch.empty(shape, dtype=dtype, device=device)
            self.tensors[key] = t
        return t[:shape[0]] if at_least else t

    def __enter__(self):
        self._prev = static_buffers.active()
        static_buffers._tls.cur = self
        return self

    def __exit__(self, *exc):
        static_buffers._tls.cur = self._prev


class fused_update:
    """Within the block, a language-only rasterizer backward of `param` (the raw _language_feature,
    the fused-activation path) also applies `optimizer`'s Adam step to it in the same pass
    (include/lsr.h lsr_backward_args.update; train.py:104 + 134-137 at N = 1), and optimizer.step()
    then leaves it alone.  The optimizer must be a langsplat_amd.optim.Adam prepared for a capture
    (its device step block; only inside a graph capture) with `param` its one parameter.  skip: its
    skip flag (the overflow flag); fill: a device pointer to another forward's record array whose
    language slots receive the updated activated feature (langsplat_amd.pipeline), or None.

    defer=True (N > 1, include/lsr.h LSR_BWD_DEFER_TAIL): the backward runs the render backward only
    and leaves the per-Gaussian language partials in its geometry buffer; partials() is that (P, 3)
    tensor, which the caller all-reduces (AVG over the ranks), then run_tail() launches the rest in
    one pass -- the gradient outputs, the Adam step and the fill (lsr_language_tail).  The backward's
    returned gradients hold their values only after run_tail()."""

    # process-wide, not thread-local: autograd runs a CUDA node's backward on its device thread, not
    # on the thread that called loss.backward()
    _cur = None

    def __init__(self, optimizer, param: torch.Tensor, skip: Optional[torch.Tensor] = None, fill: Optional[int] = None,
                 defer: bool = False):
        self.optimizer, self.param, self.skip, self.fill = optimizer, param, skip, fill
        self.defer = bool(defer)
        self.used = False
        self.pending = None  # defer: the deferred tail's arguments (and every tensor they point into)

    def partials(self) -> torch.Tensor:
        """defer: what the caller all-reduces -- the deferred backward's 3 P language partials and the
        step's skip word after them, (3 P + 1,) fp32, a view of its buffer (include/lsr.h)."""
        if self.pending is None:
            raise RuntimeError("fused_update.partials: no deferred backward ran in this block")
        return self.pending[3]

    def run_tail(self):
        """defer: lsr_language_tail on the current stream, after the caller reduced partials()."""
        if self.pending is None:
            raise RuntimeError("fused_update.run_tail: no deferred backward ran in this block")
        s, a, _keep, part, device = self.pending
        if part.numel() == 0:
            return
        with _on_device(device):
            _check(load().lsr_language_tail(ctypes.byref(s), ctypes.byref(a), _stream(device)), "lsr_language_tail")

    @staticmethod
    def active():
        return fused_update._cur

    def __enter__(self):
        self._prev = fused_update._cur
        fused_update._cur = self
        return self

    def __exit__(self, *exc):
        fused_update._cur = self._prev

    def table(self):
        """The lsr_adam_tensor of the update (the optimizer's state and group hyper-parameters)."""
        opt, p = self.optimizer, self.param
        gi = next(i for i, g in enumerate(opt.param_groups) if any(q is p for q in g["params"]))
        g = opt.param_groups[gi]
        st = opt.state[p]
        beta1, beta2 = g["betas"]
        opt._register_fused(gi)
        return LsrAdamTensor(p.numel(), p.data_ptr(), None, st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(),
                             float(g["lr"]), float(beta1), float(beta2), float(g["eps"]), opt.step_offset(p))


def output_tensor(key, shape, dtype, device) -> torch.Tensor:
    """An output tensor of the rasterizer forward: the active static_buffers' persistent one, else new."""
    st = static_buffers.active()
    if st is None:
        return torch.empty(shape, dtype=dtype, device=device)
    # a fresh alias of the persistent tensor: the autograd Function that returns it sets ITS grad_fn,
    # so the persistent tensor never keeps an autograd graph (and the parameters' AccumulateGrad
    # nodes, bound to the capture stream) alive past the step that produced it
    return st.tensor(("out", key), shape, dtype, device).detach()


# (P, W, H) -> (tile instances, super-tile entries) of this thread's last forward outside capacity mode
# (the capacities a later capture needs)
LAST_COUNTS: Dict[tuple, tuple] = {}


_SETTINGS_CACHE: Dict[int, tuple] = {}


def make_settings(rs, keep: list) -> LsrSettings:
    """lsr_settings from a GaussianRasterizationSettings (gaussian_renderer/__init__.py:37-51).

    Cached per settings object (a NamedTuple, so immutable): render() builds one per view and the
    forward and backward both convert it.  The cache holds the object, so its id stays unique."""
    hit = _SETTINGS_CACHE.get(id(rs))
    if hit is not None and hit[0] is rs:
        keep.append(hit[2])
        return hit[1]
    mine: list = []
    s = _build_settings(rs, mine)
    if len(_SETTINGS_CACHE) >= 16:
        _SETTINGS_CACHE.clear()
    _SETTINGS_CACHE[id(rs)] = (rs, s, mine)
    keep.append(mine)
    return s


def _build_settings(rs, keep: list) -> LsrSettings:
    s = LsrSettings()
    s.image_height = int(rs.image_height)
    s.image_width = int(rs.image_width)
    s.tanfovx = float(rs.tanfovx)
    s.tanfovy = float(rs.tanfovy)
    s.scale_modifier = float(rs.scale_modifier)
    s.sh_degree = int(rs.sh_degree)
    s.prefiltered = int(bool(rs.prefiltered))
    s.debug = int(bool(rs.debug))
    s.include_feature = int(bool(getattr(rs, "include_feature", False)))
    for name in ("bg", "viewmatrix", "projmatrix", "campos"):
        t = _f32c_cached(getattr(rs, name))
        keep.append(t)
        setattr(s, name, t.data_ptr())
    return s


_CONTIG_CACHE: Dict[int, tuple] = {}


def _f32c_cached(src: torch.Tensor) -> torch.Tensor:
    """_f32c of a camera tensor, reused while the source object and its version are unchanged.

    render() builds new settings every step from the same camera tensors, and the reference's
    world_view_transform is a transposed view (scene/cameras.py:47): without the cache every step
    pays a small copy kernel for it."""
    t = src.detach()
    if t.dtype == torch.float32 and t.is_contiguous():
        return t
    hit = _CONTIG_CACHE.get(id(src))
    if hit is not None and hit[0] is src and hit[1] == src._version:
        return hit[2]
    c = _f32c(t)
    if len(_CONTIG_CACHE) >= 64:
        _CONTIG_CACHE.clear()
    _CONTIG_CACHE[id(src)] = (src, src._version, c)
    return c


def rasterize_gaussians(rs, means3D, shs, colors_precomp, language_feature, opacities, scales, rotations,
                        cov3D_precomp, raw=0, shs_rest=None, visible=None, loss_target=None, loss_mask=None,
                        out_loss=None, flags=0):
    """Native forward: returns (num_rendered, color, language_feature_image, radii, geom, binning, image).

    raw / shs_rest: the fused-activation form (include/lsr.h lsr_raw_flags); shs is then
    features_dc (P,1,3) and shs_rest features_rest (P,M-1,3).  visible: optional (P,) bool tensor
    that receives radii > 0.  out_loss: optional () fp32 tensor that receives the fused
    l1_loss(lang * mask, loss_target * mask) (loss_target (3,H,W) fp32, loss_mask H*W bool)."""
    lib = load()
    device = means3D.device
    P = int(means3D.shape[0])
    H, W = int(rs.image_height), int(rs.image_width)
    keep: list = []
    s = make_settings(rs, keep)
    color = output_tensor("color", (3, H, W), torch.float32, device)
    lang = output_tensor("language", (3, H, W), torch.float32, device)
    radii = output_tensor("radii", (P,), torch.int32, device)  # preprocess writes every entry
    a = LsrForwardArgs()
    a.P = P
    a.M = int(shs.shape[1]) if shs is not None and shs.numel() > 0 else 0
    if shs_rest is not None and shs_rest.numel() > 0:
        a.M += int(shs_rest.shape[1])
        a.shs_rest = _ptr(shs_rest)
    a.raw = int(raw)
    a.flags = int(flags)
    a.means3D = _ptr(means3D)
    a.shs = _ptr(shs)
    a.colors_precomp = _ptr(colors_precomp)
    a.language_feature = _ptr(language_feature)
    a.opacities = _ptr(opacities)
    a.scales = _ptr(scales)
    a.rotations = _ptr(rotations)
    a.cov3D_precomp = _ptr(cov3D_precomp)
    a.out_color = _ptr(color)
    a.out_language_feature = _ptr(lang)
    a.radii = _ptr(radii)
    if visible is not None:
        if visible.dtype != torch.bool or visible.numel() != P or not visible.is_contiguous():
            raise ValueError("visible must be a contiguous (P,) bool tensor")
        a.visible = _ptr(visible)
    if out_loss is not None:
        if loss_target is None or tuple(loss_target.shape) != (3, H, W) or loss_target.dtype != torch.float32 \
                or not loss_target.is_contiguous():
            raise ValueError("loss_target must be a contiguous (3,H,W) fp32 tensor")
        if loss_mask is None or loss_mask.dtype != torch.bool or loss_mask.numel() != H * W \
                or not loss_mask.is_contiguous():
            raise ValueError("loss_mask must be a contiguous bool tensor of H*W elements")
        a.loss_target = _ptr(loss_target)
        a.loss_mask = _ptr(loss_mask)
        a.out_loss = _ptr(out_loss)
    cap = capacity.active()
    entries = ctypes.c_int64(0)
    ready = language_ready.active()
    if ready is not None and language_feature is not None:
        a.language_ready = ready.cuda_event
        keep.append(ready)
    a.phase = forward_phase.active()
    if cap is not None:
        a.capacity_rendered = cap.rendered
        a.capacity_entries = cap.entries
        a.overflow = _ptr(cap.overflow)
    else:
        a.out_num_entries = ctypes.pointer(entries)
    alloc = _Allocator(device)
    nr = ctypes.c_int64(0)
    with _on_device(device), alloc:
        _check(lib.lsr_forward(ctypes.byref(s), ctypes.byref(a), _ALLOC_CB, None, _stream(device), ctypes.byref(nr)),
               "lsr_forward")
    if cap is None:
        LAST_COUNTS[(P, W, H)] = (int(nr.value), int(entries.value))
    return (int(nr.value), color, lang, radii, alloc.get(LSR_BUF_GEOM), alloc.get(LSR_BUF_BINNING),
            alloc.get(LSR_BUF_IMAGE))


# LSR_ALL_GRADS=1 (or setting this to True) computes every geometry gradient even when no input
# needs one -- the reference extension's behaviour; kept for comparisons and debugging.
FORCE_GEOMETRY_GRADS = os.environ.get("LSR_ALL_GRADS", "0") == "1"


def geometry_grads_needed(needs_input_grad, geometry_inputs):
    """True if an autograd input among `geometry_inputs` (everything but means2D and the language
    feature) needs a gradient -- torch's ctx.needs_input_grad, as any autograd.Function uses it."""
    return FORCE_GEOMETRY_GRADS or any(needs_input_grad[i] for i in geometry_inputs)


def rasterize_gaussians_backward(rs, means3D, shs, colors_precomp, language_feature, scales, rotations,
                                 cov3D_precomp, radii, grad_color, grad_language, num_rendered, geom, binning,
                                 image, raw=0, shs_rest=None, opacities=None, geometry=True, grad_loss=None,
                                 flags=0, update=None):
    """Native backward: returns the gradient tensors keyed like the reference's inputs (with raw
    flags: w.r.t. the raw parameters; "shs" is then dL/dfeatures_dc and "shs_rest"
    dL/dfeatures_rest).  geometry=False (no geometry input needs a gradient): only "means2D" and
    "language_feature_precomp" are computed, the other entries are None (include/lsr.h).
    grad_loss: dL/d(the fused loss of the forward), a () device tensor, or None.  update: a
    fused_update whose Adam step the backward applies to language_feature (include/lsr.h
    lsr_backward_args.update)."""
    lib = load()
    device = means3D.device
    P = int(means3D.shape[0])
    split = shs_rest is not None and shs_rest.numel() > 0
    M_dc = int(shs.shape[1]) if shs is not None and shs.numel() > 0 else 0
    M_rest = int(shs_rest.shape[1]) if split else 0
    M = M_dc + M_rest
    keep: list = []
    s = make_settings(rs, keep)
    # every gradient output is a view of ONE allocation (one caching-allocator call per backward)
    shapes = [("means2D", (P, 3)), ("language_feature_precomp", (P, 3))]
    if geometry:
        shapes += [("colors_precomp", (P, 3)), ("opacities", (P, 1)), ("means3D", (P, 3))]
    if geometry and _ptr(cov3D_precomp) is not None:
        shapes.append(("cov3D_precomp", (P, 6)))
    if geometry and M_dc > 0:
        shapes.append(("shs", (P, M_dc, 3)))
    if geometry and split:
        shapes.append(("shs_rest", (P, M_rest, 3)))
    if geometry and _ptr(scales) is not None:
        shapes.append(("scales", (P, 3)))
    if geometry and _ptr(rotations) is not None:
        shapes.append(("rotations", (P, 4)))
    sizes = [math.prod(sh) for _, sh in shapes]
    aligned = [(n + 63) // 64 * 64 for n in sizes]  # 256-B aligned views (vector loads/stores)
    flat = torch.empty((max(sum(aligned), 1),), dtype=torch.float32, device=device)
    g = dict.fromkeys(("means2D", "colors_precomp", "language_feature_precomp", "opacities", "means3D",
                       "cov3D_precomp", "shs", "shs_rest", "scales", "rotations"))
    off = 0
    for (name, sh), n, na in zip(shapes, sizes, aligned):
        g[name] = flat[off:off + n].view(sh)
        off += na
    if P == 0:
        if update is not None and update.defer:
            update.pending = (None, None, [], torch.empty((0,), dtype=torch.float32, device=device), device)
            update.used = True
        return {k: (v.zero_() if v is not None else None) for k, v in g.items()}
    a = LsrBackwardArgs()
    a.P = P
    a.M = M
    a.num_rendered = int(num_rendered)
    a.means3D = _ptr(means3D)
    a.shs = _ptr(shs)
    a.colors_precomp = _ptr(colors_precomp)
    a.language_feature = _ptr(language_feature)
    a.opacities = _ptr(opacities)
    a.raw = int(raw)
    a.flags = int(flags)
    if split:
        a.shs_rest = _ptr(shs_rest)
        a.dL_dsh_rest = _ptr(g["shs_rest"])
    a.scales = _ptr(scales)
    a.rotations = _ptr(rotations)
    a.cov3D_precomp = _ptr(cov3D_precomp)
    a.radii = _ptr(radii)
    gc = _f32c(grad_color.detach()) if grad_color is not None else None  # None: zero colour gradient
    a.dL_dout_color = _ptr(gc)
    gl = None
    if grad_language is not None:
        gl = _f32c(grad_language.detach())
        a.dL_dout_language_feature = _ptr(gl)
    gls = None
    if grad_loss is not None:
        gls = _f32c(grad_loss.detach().reshape(1))
        a.dL_dloss = _ptr(gls)
    a.geom_buffer = _ptr(geom)
    a.binning_buffer = _ptr(binning)
    a.image_buffer = _ptr(image)
    a.dL_dmeans2D = _ptr(g["means2D"])
    a.dL_dcolors = _ptr(g["colors_precomp"])
    a.dL_dlanguage_feature = _ptr(g["language_feature_precomp"])
    a.dL_dopacity = _ptr(g["opacities"])
    a.dL_dmeans3D = _ptr(g["means3D"])
    a.dL_dcov3D = _ptr(g["cov3D_precomp"])
    a.dL_dsh = _ptr(g["shs"])
    a.dL_dscales = _ptr(g["scales"])
    a.dL_drotations = _ptr(g["rotations"])
    if update is not None:
        tab = update.table()
        keep.append(tab)
        a.update = ctypes.pointer(tab)
        a.update_step_dev = ctypes.c_void_p(update.optimizer._step_dev.data_ptr())
        a.update_skip = _ptr(update.skip)
        a.fill_record = None if update.fill is None else ctypes.c_void_p(int(update.fill))
        update.used = True
        if update.defer:
            a.flags |= BWD_DEFER_TAIL
    alloc = _Allocator(device)
    with _on_device(device), alloc:
        _check(lib.lsr_backward(ctypes.byref(s), ctypes.byref(a), _ALLOC_CB, None, _stream(device)), "lsr_backward")
    if update is not None and update.defer:
        # the records' language partials and the skip word: the first 3 P + 1 floats of grad_records
        off = state_layout(P, int(rs.image_width), int(rs.image_height), int(num_rendered))["grad_records"]
        part = geom[off:off + 4 * (3 * P + 1)].view(torch.float32)
        # every tensor the deferred launch's pointers reach stays alive with it
        keep += [flat, geom, binning, image, radii, language_feature, update.skip, gl, gls, gc, means3D]
        update.pending = (s, a, keep, part, device)
    return g


def densification_stats(radii, dmeans2D, max_radii2D=None, xyz_gradient_accum=None, denom=None):
    """train.py:125-126 in one kernel (include/lsr.h lsr_densification_stats), in place: for radii > 0,
    max_radii2D = max(max_radii2D, radii), xyz_gradient_accum += ||dmeans2D[:, :2]||, denom += 1."""
    lib = load()
    P = int(radii.shape[0])
    outs = []
    for t, shape in ((max_radii2D, (P,)), (xyz_gradient_accum, (P, 1)), (denom, (P, 1))):
        if t is not None and (t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != P):
            raise ValueError(f"densification_stats: expected a contiguous fp32 tensor of {shape}")
        outs.append(_ptr(t))
    if radii.dtype != torch.int32 or not radii.is_contiguous():
        raise ValueError("densification_stats: radii must be a contiguous int32 tensor")
    g = _f32c(dmeans2D.detach())
    if tuple(g.shape) != (P, 3):
        raise ValueError("densification_stats: dmeans2D must be (P, 3)")
    with _on_device(radii.device):
        _check(lib.lsr_densification_stats(P, _ptr(radii), _ptr(g), *outs, _stream(radii.device)),
               "lsr_densification_stats")


def fill_language(language_feature: torch.Tensor, raw: int, radii: torch.Tensor, record_ptr: int):
    """The language slots of a geometry-phase forward's render records from the parameter, on the
    current stream (include/lsr.h lsr_fill_language)."""
    P = int(radii.shape[0])
    lf = _f32c(language_feature.detach())
    if tuple(lf.shape) != (P, 3) or radii.dtype != torch.int32 or not radii.is_contiguous():
        raise ValueError("fill_language: a (P, 3) feature and the (P,) int32 radii of the same forward")
    with _on_device(lf.device):
        _check(load().lsr_fill_language(P, _ptr(lf), int(raw), _ptr(radii), ctypes.c_void_p(int(record_ptr)),
                                        _stream(lf.device)), "lsr_fill_language")


def mark_visible(means3D, viewmatrix, projmatrix):
    lib = load()
    device = means3D.device
    P = int(means3D.shape[0])
    vis = torch.zeros((P,), dtype=torch.uint8, device=device)
    m = _f32c(means3D.detach())
    v = _f32c(viewmatrix.detach())
    p = _f32c(projmatrix.detach())
    with _on_device(device):
        _check(lib.lsr_mark_visible(P, _ptr(m), _ptr(v), _ptr(p), _ptr(vis), _stream(device)), "lsr_mark_visible")
    return vis.bool()


def state_layout(P: int, W: int, H: int, num_rendered: int) -> Dict[str, int]:
    lay = LsrStateLayout()
    _check(load().lsr_state_layout_of(P, W, H, num_rendered, ctypes.byref(lay)), "lsr_state_layout_of")
    return {name: int(getattr(lay, name)) for name, _ in LsrStateLayout._fields_}


def profile_enable(on: bool = True, stages=None, every: int = 1):
    """Start (clearing) / stop the per-stage HIP-event profiler; `stages` restricts it to those
    stage names (lsr_profile_select), `every` > 1 records only every every-th selected launch
    (lsr_profile_sample)."""
    lib = load()
    lib.lsr_profile_select(",".join(stages).encode() if stages else None)
    _check(lib.lsr_profile_sample(int(every)), "lsr_profile_sample")
    lib.lsr_profile_enable(1 if on else 0)


def profile_report() -> Dict[str, Dict[str, float]]:
    """{stage: {"launches": n, "total_ms": t, "avg_ms": t / n}} (synchronises recorded events)."""
    lib = load()
    n = lib.lsr_profile_report(None, 0)
    arr = (LsrKernelStat * max(n, 1))()
    n = lib.lsr_profile_report(arr, n)
    out = {}
    for i in range(n):
        k = arr[i].name.decode()
        out[k] = {"launches": int(arr[i].launches), "total_ms": float(arr[i].total_ms),
                  "avg_ms": float(arr[i].total_ms) / max(int(arr[i].launches), 1)}
    return out


def debug_render_stats():
    """Counters of the LSR_RENDER_STATS=1 backward (include/lsr.h lsr_debug_render_stats); clears them."""
    arr = (ctypes.c_uint64 * 73)()
    _check(load().lsr_debug_render_stats(arr, 73), "lsr_debug_render_stats")
    v = list(arr)
    return {"entries": v[0], "power_hit": v[1], "alpha_hit": v[2], "lanes_hit": v[3], "barrier_slots": v[4],
            "batches": v[6], "hist": v[8:8 + 65]}


def debug_render_timeline(kernel, n):
    """Per-workgroup timeline of the LSR_RENDER_STATS=1 render kernels (kernel 0 forward, 1 backward;
    include/lsr.h lsr_debug_render_timeline): for workgroups < n, dicts with start, end, tile,
    slot and (forward) the load / compact / walk ticks, the batch count, the first batch's load ticks and its milestones (ticks after the start: begin,
    ranges loaded, first barrier, ids loaded, records gathered, load phase done)."""
    W = 11
    arr = (ctypes.c_uint32 * (W * n))()
    _check(load().lsr_debug_render_timeline(kernel, arr, n), "lsr_debug_render_timeline")
    v = list(arr)
    out = []
    for i in range(n):
        r = v[W * i:W * i + W]
        out.append({"start": r[0], "end": r[1], "tile": r[2] if r[2] < 2 ** 31 else r[2] - 2 ** 32, "slot": r[3],
                    "load": r[4], "compact": r[5], "walk": r[6], "batches": r[7] & 0xFFFF,
                    "first_load": r[7] >> 16,
                    "first_marks": [r[8] & 0xFFFF, r[8] >> 16, r[9] & 0xFFFF, r[9] >> 16, r[10] & 0xFFFF, r[10] >> 16]})
    return out

