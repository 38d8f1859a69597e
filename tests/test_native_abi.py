"""C-ABI library: loads without a GPU, exports every entry point include/lsr.h declares, and its
Python front-end enforces the reference's API contract (gaussian_renderer/__init__.py:37-105)."""
import ctypes
import os
import re

import pytest
import torch

from langsplat_amd import _native
from langsplat_amd.rasterizer import GaussianRasterizationSettings, GaussianRasterizer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_functions():
    src = open(os.path.join(ROOT, "include", "lsr.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(lsr_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_expected_entry_points():
    names = _declared_functions()
    for n in ("lsr_forward", "lsr_backward", "lsr_mark_visible", "lsr_last_error", "lsr_abi_version"):
        assert n in names


def test_library_loads_and_exports_every_declared_symbol():
    lib = _native.load()
    for name in _declared_functions():
        assert hasattr(lib, name), name
        assert name in _native.SIGNATURES, f"ctypes binding misses {name}"
    assert lib.lsr_abi_version() == _native.ABI_VERSION == 17


def test_header_constants_match_the_python_side():
    hdr = open(os.path.join(ROOT, "include", "lsr.h")).read()
    assert int(re.search(r"#define LSR_ABI_VERSION (\d+)", hdr).group(1)) == _native.ABI_VERSION
    assert int(re.search(r"#define LSR_ADAM_STEP_WORDS (\d+)", hdr).group(1)) == _native.ADAM_STEP_WORDS
    assert int(re.search(r"#define LSR_ADAM_WORD_SKIPPED (\d+)", hdr).group(1)) == _native.ADAM_WORD_SKIPPED
    assert int(re.search(r"#define LSR_ADAM_WORD_LR (\d+)", hdr).group(1)) == _native.ADAM_WORD_LR
    # 16 lr words after the skipped count fit the block
    assert _native.ADAM_WORD_LR + 16 <= _native.ADAM_STEP_WORDS
    fwd = re.search(r"enum lsr_forward_flags \{([^}]*)\}", hdr).group(1)
    vals = dict((k.strip(), int(v)) for k, v in (e.split("=") for e in fwd.split(",")))
    assert vals == {"LSR_FWD_ZERO_GRAD_RECORDS": _native.FWD_ZERO_GRAD_RECORDS,
                    "LSR_FWD_NO_COLOR_GRAD": _native.FWD_NO_COLOR_GRAD,
                    "LSR_FWD_NO_BACKWARD": _native.FWD_NO_BACKWARD}


def test_sizes_and_layout_are_consistent():
    lib = _native.load()
    P, W, H, R = 1000, 100, 70, 12345
    lay = _native.state_layout(P, W, H, R)
    assert lay["record"] % 16 == 0 and lay["record"] + 48 * P <= lib.lsr_geom_bytes(P, W, H)
    assert lay["n_contrib"] + 4 * W * H <= lib.lsr_image_bytes(W, H)
    assert lay["point_list"] + 4 * R <= lib.lsr_binning_bytes(W, H, R)
    assert lib.lsr_backward_bytes(P) == 64 * P
    assert lib.lsr_geom_bytes(2 * P, W, H) > lib.lsr_geom_bytes(P, W, H)
    # the geometry buffer carries one fused-loss word per tile: it grows with the image
    assert lib.lsr_geom_bytes(P, 1920, 1080) > lib.lsr_geom_bytes(P, W, H)
    # the language step's gradient records (ABI 16: the deferred tail's all-reduce reads their first 3 P
    # floats as a (P, 3) view): 4-B aligned floats inside the geometry buffer
    assert lay["grad_records"] % 256 == 0 and lay["grad_records"] + 20 * P <= lib.lsr_geom_bytes(P, W, H)


def test_invalid_arguments_report_errors_without_gpu():
    lib = _native.load()
    assert lib.lsr_state_layout_of(-1, 10, 10, 0, None) != 0
    assert "invalid" in _native.last_error()
    assert lib.lsr_mark_visible(-5, None, None, None, None, None) != 0


def test_forward_flag_and_phase_validation_without_gpu():
    """lsr_forward refuses an unknown flag, and a forward phase (include/lsr.h lsr_forward_phase)
    outside capacity mode, before any device work (dummy non-null pointers, never dereferenced)."""
    import ctypes
    lib = _native.load()
    dummy = ctypes.c_void_p(256)
    s = _native.LsrSettings()
    s.image_height, s.image_width, s.tanfovx, s.tanfovy, s.sh_degree = 8, 8, 0.5, 0.5, 0
    s.bg = s.viewmatrix = s.projmatrix = s.campos = dummy
    nr = ctypes.c_int64(0)

    def call(**kw):
        a = _native.LsrForwardArgs()
        a.P, a.M = 4, 1
        a.means3D = a.shs = a.opacities = a.scales = a.rotations = dummy
        a.out_color = a.out_language_feature = a.radii = dummy
        for k, v in kw.items():
            setattr(a, k, v)
        return lib.lsr_forward(ctypes.byref(s), ctypes.byref(a), _native._ALLOC_CB, None, None, ctypes.byref(nr))

    assert call(flags=8) != 0 and "unknown flag" in _native.last_error()
    assert call(phase=_native.forward_phase.GEOMETRY) != 0 and "phase" in _native.last_error()
    assert call(phase=4, capacity_rendered=16, capacity_entries=16) != 0 and "phase" in _native.last_error()
    assert call(phase=_native.forward_phase.COMPOSITE_FILLED) != 0 and "phase" in _native.last_error()
    assert call(phase=_native.forward_phase.COMPOSITE, capacity_rendered=16, capacity_entries=16,
                language_ready=dummy) != 0 and "phase" in _native.last_error()


def test_backward_fused_update_validation_without_gpu():
    """lsr_backward_args.update (ABI 12, the language step's Adam fused into the epilogue) is refused
    before any device work unless it is the language-only backward of the raw feature it updates; the
    update's companions without an update are refused too (dummy pointers, never dereferenced)."""
    import ctypes
    lib = _native.load()
    dummy = ctypes.c_void_p(256)
    s = _native.LsrSettings()
    s.image_height, s.image_width, s.tanfovx, s.tanfovy, s.sh_degree, s.include_feature = 8, 8, 0.5, 0.5, 0, 1
    s.bg = s.viewmatrix = s.projmatrix = s.campos = dummy
    P = 4

    def call(update_param=256, geometry=False, raw=_native.RAW_LANGUAGE, with_update=True, **kw):
        a = _native.LsrBackwardArgs()
        a.P, a.M, a.num_rendered = P, 1, 16
        a.means3D = a.shs = a.opacities = a.scales = a.rotations = a.radii = dummy
        a.language_feature = ctypes.c_void_p(256)
        a.geom_buffer = a.binning_buffer = a.image_buffer = dummy
        a.dL_dmeans2D = a.dL_dlanguage_feature = dummy
        a.raw = raw
        if geometry:
            a.dL_dcolors = a.dL_dopacity = a.dL_dmeans3D = a.dL_dsh = a.dL_dscales = a.dL_drotations = dummy
        t = _native.LsrAdamTensor(3 * P, update_param, None, 512, 768, 0.01, 0.9, 0.999, 1e-15, 0)
        if with_update:
            a.update = ctypes.pointer(t)
            a.update_step_dev = dummy
        for k, v in kw.items():
            setattr(a, k, v)
        return lib.lsr_backward(ctypes.byref(s), ctypes.byref(a), _native._ALLOC_CB, None, None)

    assert call(geometry=True) != 0 and "fused update" in _native.last_error()
    assert call(raw=0) != 0 and "fused update" in _native.last_error()
    assert call(update_param=1024) != 0 and "fused update" in _native.last_error()
    assert call(dL_dout_color=dummy) != 0 and "fused update" in _native.last_error()
    assert call(update_step_dev=None) != 0 and "fused update" in _native.last_error()
    assert call(with_update=False, fill_record=dummy) != 0 and "need update" in _native.last_error()
    # LSR_BWD_DEFER_TAIL (ABI 16) is a form of the fused update
    assert call(with_update=False, flags=_native.BWD_DEFER_TAIL) != 0 and "needs update" in _native.last_error()
    assert call(geometry=True, flags=_native.BWD_DEFER_TAIL) != 0 and "fused update" in _native.last_error()

    def tail(**kw):
        a = _native.LsrBackwardArgs()
        a.P, a.M, a.num_rendered = P, 1, 16
        a.radii = a.geom_buffer = dummy
        a.language_feature = ctypes.c_void_p(256)
        a.dL_dlanguage_feature = dummy
        a.raw = _native.RAW_LANGUAGE
        t = _native.LsrAdamTensor(3 * P, 256, None, 512, 768, 0.01, 0.9, 0.999, 1e-15, 0)
        a.update = ctypes.pointer(t)
        a.update_step_dev = dummy
        for k, v in kw.items():
            setattr(a, k, v)
        return lib.lsr_language_tail(ctypes.byref(s), ctypes.byref(a), None)

    assert lib.lsr_language_tail(None, None, None) != 0 and "null" in _native.last_error()
    assert tail(update=None) != 0 and "fused update" in _native.last_error()
    assert tail(raw=0) != 0 and "fused update" in _native.last_error()
    assert tail(dL_dlanguage_feature=None) != 0 and "fused update" in _native.last_error()
    assert tail(geom_buffer=None) != 0 and "forward state" in _native.last_error()
    assert tail(fill_record=ctypes.c_void_p(264)) != 0 and "16-byte" in _native.last_error()


def test_spin_limit_knob_round_trips_without_gpu():
    lib = _native.load()
    old = lib.lsr_debug_set_spin_limit(7)
    assert lib.lsr_debug_set_spin_limit(old) == 7
    assert old == 1 << 24


def _settings(device="cpu", include_feature=True):
    return GaussianRasterizationSettings(
        image_height=8, image_width=8, tanfovx=0.5, tanfovy=0.5, bg=torch.zeros(3, device=device),
        scale_modifier=1.0, viewmatrix=torch.eye(4, device=device), projmatrix=torch.eye(4, device=device),
        sh_degree=0, campos=torch.zeros(3, device=device), prefiltered=False, debug=False,
        include_feature=include_feature)


def test_settings_namedtuple_has_the_13_reference_fields():
    s = _settings()
    assert GaussianRasterizationSettings._fields == (
        "image_height", "image_width", "tanfovx", "tanfovy", "bg", "scale_modifier", "viewmatrix", "projmatrix",
        "sh_degree", "campos", "prefiltered", "debug", "include_feature")
    assert s.include_feature is True


def test_exactly_one_of_validation():
    r = GaussianRasterizer(_settings())
    m = torch.zeros((4, 3))
    o = torch.ones((4, 1))
    with pytest.raises(Exception, match="exactly one of either SHs|excatly one of either SHs"):
        r(means3D=m, means2D=m, opacities=o, scales=m, rotations=torch.zeros((4, 4)))
    with pytest.raises(Exception, match="SHs or precomputed colors"):
        r(means3D=m, means2D=m, opacities=o, shs=torch.zeros((4, 1, 3)), colors_precomp=m, scales=m,
          rotations=torch.zeros((4, 4)))
    with pytest.raises(Exception, match="scale/rotation pair or precomputed 3D covariance"):
        r(means3D=m, means2D=m, opacities=o, colors_precomp=m)
    with pytest.raises(Exception, match="scale/rotation pair or precomputed 3D covariance"):
        r(means3D=m, means2D=m, opacities=o, colors_precomp=m, scales=m, rotations=torch.zeros((4, 4)),
          cov3D_precomp=torch.zeros((4, 6)))


def test_cpu_tensors_are_rejected_loudly():
    """No silent CPU fallback in the product path."""
    r = GaussianRasterizer(_settings())
    m = torch.zeros((4, 3))
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        r(means3D=m, means2D=m, opacities=torch.ones((4, 1)), colors_precomp=m, scales=m,
          rotations=torch.zeros((4, 4)))


def test_drop_in_module_name():
    import diff_gaussian_rasterization as dgr
    assert dgr.GaussianRasterizer is GaussianRasterizer
    assert dgr.GaussianRasterizationSettings is GaussianRasterizationSettings


def test_ctypes_struct_layouts_match_header(tmp_path):
    """Every ctypes mirror in _native.py has the C header's field offsets and sizes (gcc on lsr.h)."""
    import subprocess
    structs = {"lsr_settings": _native.LsrSettings, "lsr_forward_args": _native.LsrForwardArgs,
               "lsr_backward_args": _native.LsrBackwardArgs, "lsr_state_layout": _native.LsrStateLayout,
               "lsr_kernel_stat": _native.LsrKernelStat}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "lsr.h"', "int main(void) {"]
    for cname, cls in structs.items():
        lines.append(f'printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for f in cls._fields_:
            lines.append(f'printf("{cname} {f[0]} %zu\\n", offsetof({cname}, {f[0]}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    subprocess.run(["gcc", "-I", inc, str(src), "-o", str(exe)], check=True)
    got = {}
    for ln in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        s, f, v = ln.split()
        got[(s, f)] = int(v)
    for cname, cls in structs.items():
        assert got[(cname, "sizeof")] == ctypes.sizeof(cls), cname
        for f in cls._fields_:
            assert got[(cname, f[0])] == getattr(cls, f[0]).offset, (cname, f[0])


def test_optim_adam_refuses_cpu_parameters():
    from langsplat_amd.optim import Adam
    p = torch.zeros(4, requires_grad=True)
    p.grad = torch.ones(4)
    opt = Adam([p], lr=0.1)
    with pytest.raises(RuntimeError, match="no CPU path"):
        opt.step()


def test_graph_launch_refuses_invalid_arguments_without_a_gpu():
    """lsr_graph_launch (ABI 17) checks its arguments before any HIP call: no executable, a negative
    wait count, or waits without an array are LSR_ERR_INVALID with a message."""
    lib = _native.load()
    assert lib.lsr_graph_launch(None, None, None, 0, None) == 1
    assert b"lsr_graph_launch" in lib.lsr_last_error()
    dummy = ctypes.c_void_p(1)
    assert lib.lsr_graph_launch(dummy, None, None, -1, None) == 1
    assert lib.lsr_graph_launch(dummy, None, None, 2, None) == 1
