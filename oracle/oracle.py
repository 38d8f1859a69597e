"""ctypes front-end of the CPU oracle (oracle/lsr_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, always as the checker -- never by the product path (langsplat_amd/,
diff_gaussian_rasterization/), which must fail loudly rather than fall back to this.

The oracle restates the published 3DGS rasterizer that submodules/langsplat-rasterization
forks (the submodule itself is absent from /root/reference).  Its
interface mirrors the reference call site gaussian_renderer/__init__.py:96-105.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liblsr_oracle.so")
_lib = None

_f32p = ctypes.POINTER(ctypes.c_float)


class _Settings(ctypes.Structure):
    _fields_ = [
        ("image_height", ctypes.c_int32),
        ("image_width", ctypes.c_int32),
        ("tanfovx", ctypes.c_float),
        ("tanfovy", ctypes.c_float),
        ("scale_modifier", ctypes.c_float),
        ("sh_degree", ctypes.c_int32),
        ("include_feature", ctypes.c_int32),
        ("prefiltered", ctypes.c_int32),
        ("bg", ctypes.c_float * 3),
        ("viewmatrix", ctypes.c_float * 16),
        ("projmatrix", ctypes.c_float * 16),
        ("campos", ctypes.c_float * 3),
        ("form", ctypes.c_int32),
    ]

# arithmetic forms of lsr_oracle.c ("Upstream forms"): KERNEL is the kernels' operation sequence
# (the bit-exact contract); UPSTREAM / UPSTREAM_FMA evaluate the published rasterizer's source
# expressions, without / with nvcc-style multiply-add contraction
FORM_KERNEL, FORM_UPSTREAM, FORM_UPSTREAM_FMA = 0, 1, 2


def build(force: bool = False) -> str:
    """Compile the oracle with its Makefile (gcc, -ffp-contract=off)."""
    src = os.path.join(_HERE, "lsr_oracle.c")
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE, "liblsr_oracle.so"], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        L.lso_forward.restype = ctypes.c_void_p
        L.lso_forward.argtypes = [ctypes.POINTER(_Settings), ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 11
        L.lso_backward.restype = None
        L.lso_backward.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 11
        L.lso_num_rendered.restype = ctypes.c_int64
        L.lso_num_rendered.argtypes = [ctypes.c_void_p]
        L.lso_get.restype = ctypes.c_int64
        L.lso_get.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]
        L.lso_free.restype = None
        L.lso_free.argtypes = [ctypes.c_void_p]
        L.lso_expf.restype = ctypes.c_float
        L.lso_expf.argtypes = [ctypes.c_float]
        L.lso_expf_render.restype = ctypes.c_float
        L.lso_expf_render.argtypes = [ctypes.c_float]
        L.lso_sh_eval.restype = None
        L.lso_sh_eval.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.lso_sh_backward.restype = None
        L.lso_sh_backward.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 5
        L.lso_cov3d.restype = None
        L.lso_cov3d.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p]
        L.lso_act_expf.restype = ctypes.c_float
        L.lso_act_expf.argtypes = [ctypes.c_float]
        L.lso_activate.restype = None
        L.lso_activate.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 8
        L.lso_activate_backward.restype = None
        L.lso_activate_backward.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 12
        L.lso_num_threads.restype = ctypes.c_int
        L.lso_num_threads.argtypes = []
        L.lso_knn_mean_dist3.restype = None
        L.lso_knn_mean_dist3.argtypes = [ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
        L.lso_cov3d_backward.restype = None
        L.lso_cov3d_backward.argtypes = [ctypes.c_void_p, ctypes.c_float] + [ctypes.c_void_p] * 4
        _lib = L
    return _lib


def _np(x, shape=None):
    """float32 C-contiguous numpy copy of a tensor/array (or None)."""
    if x is None:
        return None
    if hasattr(x, "detach"):
        x = x.detach().cpu().numpy()
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float32))
    if shape is not None:
        a = a.reshape(shape)
    return a


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def make_settings(s, form: int = FORM_KERNEL) -> _Settings:
    """From a GaussianRasterizationSettings-like object (fields of gaussian_renderer/__init__.py:37-51)."""
    out = _Settings()
    out.form = int(form)
    out.image_height = int(s.image_height)
    out.image_width = int(s.image_width)
    out.tanfovx = float(s.tanfovx)
    out.tanfovy = float(s.tanfovy)
    out.scale_modifier = float(s.scale_modifier)
    out.sh_degree = int(s.sh_degree)
    out.include_feature = int(bool(s.include_feature))
    out.prefiltered = int(bool(s.prefiltered))
    out.bg[:] = _np(s.bg, (3,)).tolist()
    out.viewmatrix[:] = _np(s.viewmatrix, (16,)).tolist()
    out.projmatrix[:] = _np(s.projmatrix, (16,)).tolist()
    out.campos[:] = _np(s.campos, (3,)).tolist()
    return out


class OracleRun:
    """One forward pass; keeps the oracle state for backward() and state inspection."""

    _STATE_DTYPES = {
        "depth": (np.float32, 1), "xy": (np.float32, 2), "conic_opacity": (np.float32, 4),
        "rgb": (np.float32, 3), "tiles_touched": (np.uint32, 1), "clamped": (np.uint8, 3),
    }

    def __init__(self, settings, means3D, opacities, shs=None, colors_precomp=None,
                 language_feature_precomp=None, scales=None, rotations=None, cov3D_precomp=None,
                 form=FORM_KERNEL):
        L = lib()
        self.settings = settings
        self.form = int(form)
        st = make_settings(settings, form)
        self._st = st
        H, W = st.image_height, st.image_width
        self.H, self.W = H, W
        means = _np(means3D, (-1, 3))
        P = means.shape[0]
        self.P = P
        self.M = 0
        self.shs = None
        if shs is not None:
            self.shs = _np(shs)
            self.M = int(self.shs.shape[1]) if self.shs.ndim == 3 else int(self.shs.size // max(3 * P, 1))
            self.shs = self.shs.reshape(P, self.M, 3)
        self.colors = _np(colors_precomp, (P, 3)) if colors_precomp is not None else None
        lang = language_feature_precomp
        self.lang = None
        if lang is not None and np.asarray(_np(lang)).size == 3 * P and P > 0:
            self.lang = _np(lang, (P, 3))
        self.opac = _np(opacities, (P,))
        self.scales = _np(scales, (P, 3)) if scales is not None else None
        self.rots = _np(rotations, (P, 4)) if rotations is not None else None
        self.cov = _np(cov3D_precomp, (P, 6)) if cov3D_precomp is not None else None
        self.color = np.zeros((3, H, W), np.float32)
        self.language = np.zeros((3, H, W), np.float32)
        self.radii = np.zeros((P,), np.int32)
        self.means = means
        self._h = L.lso_forward(ctypes.byref(st), P, self.M, _ptr(means), _ptr(self.shs),
                                _ptr(self.colors), _ptr(self.lang), _ptr(self.opac),
                                _ptr(self.scales), _ptr(self.rots), _ptr(self.cov),
                                _ptr(self.color), _ptr(self.language), _ptr(self.radii))
        self.num_rendered = int(L.lso_num_rendered(self._h))
        self.gx = (W + 15) // 16
        self.gy = (H + 15) // 16

    def get(self, name):
        L = lib()
        P, HW, T = self.P, self.H * self.W, self.gx * self.gy
        if name in self._STATE_DTYPES:
            dt, k = self._STATE_DTYPES[name]
            out = np.zeros((P, k) if k > 1 else (P,), dt)
        elif name == "point_list":
            out = np.zeros((self.num_rendered,), np.uint32)
        elif name == "ranges":
            out = np.zeros((T, 2), np.uint32)
        elif name == "final_T":
            out = np.zeros((self.H, self.W), np.float32)
        elif name == "n_contrib":
            out = np.zeros((self.H, self.W), np.uint32)
        else:
            raise KeyError(name)
        n = L.lso_get(self._h, name.encode(), out.ctypes.data_as(ctypes.c_void_p))
        assert n == out.nbytes, (name, n, out.nbytes)
        return out

    @property
    def blends(self) -> int:
        """Sum over pixels of n_contrib (SURVEY.md §8d unit of work)."""
        return int(self.get("n_contrib").astype(np.int64).sum())

    def backward(self, grad_color, grad_language=None):
        """Returns the rasterizer gradients in the reference's naming."""
        L = lib()
        P, M = self.P, self.M
        gc = _np(grad_color, (3, self.H, self.W))
        gl = _np(grad_language, (3, self.H, self.W)) if grad_language is not None else None
        out = {
            "means2D": np.zeros((P, 3), np.float32),
            "colors_precomp": np.zeros((P, 3), np.float32),
            "language_feature_precomp": np.zeros((P, 3), np.float32),
            "opacities": np.zeros((P, 1), np.float32),
            "means3D": np.zeros((P, 3), np.float32),
            "cov3D_precomp": np.zeros((P, 6), np.float32),
            "shs": np.zeros((P, max(M, 0), 3), np.float32),
            "scales": np.zeros((P, 3), np.float32),
            "rotations": np.zeros((P, 4), np.float32),
        }
        L.lso_backward(self._h, _ptr(gc), _ptr(gl), _ptr(out["means2D"]), _ptr(out["colors_precomp"]),
                       _ptr(out["language_feature_precomp"]), _ptr(out["opacities"]), _ptr(out["means3D"]),
                       _ptr(out["cov3D_precomp"]), _ptr(out["shs"]) if M > 0 else None,
                       _ptr(out["scales"]) if self.cov is None else None,
                       _ptr(out["rotations"]) if self.cov is None else None)
        return out

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib is not None:
            _lib.lso_free(h)
            self._h = None


def forward(settings, **kw) -> OracleRun:
    return OracleRun(settings, **kw)


def num_threads() -> int:
    """Threads of the oracle's OpenMP loops (OMP_NUM_THREADS, else the host's cores)."""
    return int(lib().lso_num_threads())


def expf(x: float) -> float:
    return float(lib().lso_expf(float(x)))


def expf_render(x: float) -> float:
    """The compositing loops' exp (lsr_oracle.c lso_expf_render; x >= -20)."""
    return float(lib().lso_expf_render(float(x)))


def sh_eval(deg: int, sh: np.ndarray, dirs: np.ndarray) -> np.ndarray:
    """sh: (N, K, 3) coefficient-major like GaussianModel.get_features; dirs: (N, 3) unit."""
    L = lib()
    sh = _np(sh)
    dirs = _np(dirs)
    N = dirs.shape[0]
    out = np.zeros((N, 3), np.float32)
    for i in range(N):
        L.lso_sh_eval(deg, _ptr(sh[i]), _ptr(dirs[i]), _ptr(out[i]))
    return out


def sh_backward(deg: int, sh: np.ndarray, dir_orig: np.ndarray, dL_drgb: np.ndarray):
    """Returns (dL/dsh (N,K,3), dL/d(unnormalised direction) (N,3))."""
    L = lib()
    sh = _np(sh)
    dir_orig = _np(dir_orig)
    g = _np(dL_drgb)
    N, K = sh.shape[0], sh.shape[1]
    dsh = np.zeros((N, K, 3), np.float32)
    dm = np.zeros((N, 3), np.float32)
    for i in range(N):
        L.lso_sh_backward(deg, K, _ptr(sh[i]), _ptr(dir_orig[i]), _ptr(g[i]), _ptr(dsh[i]), _ptr(dm[i]))
    return dsh, dm


def cov3d(scales: np.ndarray, mod: float, rots: np.ndarray) -> np.ndarray:
    L = lib()
    scales, rots = _np(scales), _np(rots)
    out = np.zeros((scales.shape[0], 6), np.float32)
    for i in range(scales.shape[0]):
        L.lso_cov3d(_ptr(scales[i]), float(mod), _ptr(rots[i]), _ptr(out[i]))
    return out


def cov3d_backward(scales, mod, rots, dcov):
    L = lib()
    scales, rots, dcov = _np(scales), _np(rots), _np(dcov)
    N = scales.shape[0]
    ds = np.zeros((N, 3), np.float32)
    dr = np.zeros((N, 4), np.float32)
    for i in range(N):
        L.lso_cov3d_backward(_ptr(scales[i]), float(mod), _ptr(rots[i]), _ptr(dcov[i]), _ptr(ds[i]), _ptr(dr[i]))
    return ds, dr


RAW_OPACITY, RAW_SCALES, RAW_ROTATIONS, RAW_LANGUAGE = 1, 2, 4, 8
RAW_ALL = RAW_OPACITY | RAW_SCALES | RAW_ROTATIONS | RAW_LANGUAGE


def activate(raw, opacity=None, scales=None, rotations=None, language=None):
    """lso_activate: GaussianModel's activations of the raw parameters (float32 numpy out).
    Returns (opacity, scales, rotations, language) with None for absent inputs."""
    L = lib()
    ins = [None if x is None else _np(x) for x in (opacity, scales, rotations, language)]
    P = next(x.shape[0] for x in ins if x is not None)
    outs = [None if x is None else np.zeros_like(x) for x in ins]
    L.lso_activate(P, int(raw), *[_ptr(x) if x is not None else None for x in ins],
                   *[_ptr(x) if x is not None else None for x in outs])
    return tuple(outs)


def activate_backward(raw, raw_inputs, grads):
    """lso_activate_backward: gradients w.r.t. activated tensors -> w.r.t. the raw tensors.
    raw_inputs, grads: 4-tuples (opacity, scales, rotations, language) with None for absent."""
    L = lib()
    ins = [None if x is None else _np(x) for x in raw_inputs]
    gs = [None if g is None else _np(g) for g in grads]
    P = next(x.shape[0] for x in ins if x is not None)
    outs = [None if x is None else np.zeros_like(x) for x in ins]
    p = lambda x: _ptr(x) if x is not None else None  # noqa: E731
    L.lso_activate_backward(P, int(raw), *[p(x) for x in ins], *[p(g) for g in gs], *[p(o) for o in outs])
    return tuple(outs)


def knn_mean_dist3(points) -> np.ndarray:
    """lso_knn_mean_dist3: brute-force distCUDA2 (mean squared distance to the 3 nearest others)."""
    p = _np(points)
    out = np.zeros((p.shape[0],), np.float32)
    lib().lso_knn_mean_dist3(p.shape[0], _ptr(p), _ptr(out))
    return out
