"""MSD vs LSD depth order at C5 (measurement aid for DESIGN.md §8; profiles/r05_c5_msd_vs_lsd.txt):

    python3 tools/c5_msd_check.py

Renders the C5 forward twice, once with the LSD depth order (LSR_DEPTH_LSD=1) and once with the MSD
bucket sort forced on (LSR_MSD_MAX_KEYS=4000000), prints each one's per-kernel times, and compares
the images, tile ranges, point list, final T and contributor counts for bit equality.
"""
import os, sys, time
sys.path.insert(0, os.getcwd())
import torch, numpy as np
from langsplat_amd import _native
from langsplat_amd.synthetic import CONFIGS, make_cameras, make_gaussians, activated_inputs
from tests.scenes import settings_for
from tests.test_gpu_parity import state
c = CONFIGS["C5"]; P, W, H = c["P"], c["width"], c["height"]
g = make_gaussians(P, seed=0)
cam = make_cameras(c["views"], W, H)[0]
st = settings_for(cam, sh_degree=3)
dev = "cuda"
from tests.scenes import to_device
with torch.no_grad():
    inp = activated_inputs(g)
std, ind = to_device(st, {k: v for k, v in inp.items()}, dev)
args = (ind["means3D"], ind["shs"], None, ind["language_feature_precomp"], ind["opacities"], ind["scales"], ind["rotations"], None)
outs = {}
for mode in ("lsd", "msd"):
    if mode == "lsd":
        os.environ["LSR_DEPTH_LSD"] = "1"; os.environ.pop("LSR_MSD_MAX_KEYS", None)
    else:
        os.environ.pop("LSR_DEPTH_LSD", None); os.environ["LSR_MSD_MAX_KEYS"] = "4000000"
    out = _native.rasterize_gaussians(std, *args, flags=_native.FWD_ZERO_GRAD_RECORDS)
    torch.cuda.synchronize()
    nr = out[0]
    s = state((nr, None, None, None, out[4], out[5], out[6]), P, W, H)
    outs[mode] = (out[1].cpu().numpy(), out[2].cpu().numpy(), s)
    for _ in range(3):
        _native.rasterize_gaussians(std, *args, flags=_native.FWD_ZERO_GRAD_RECORDS)
    torch.cuda.synchronize()
    _native.profile_enable(True)
    for _ in range(10):
        _native.rasterize_gaussians(std, *args, flags=_native.FWD_ZERO_GRAD_RECORDS)
    torch.cuda.synchronize()
    _native.profile_enable(False)
    rep = _native.profile_report()
    print(mode, "num_rendered", nr, {k: round(v["avg_ms"] * 1e3, 1) for k, v in rep.items()}, flush=True)
a, b = outs["lsd"], outs["msd"]
print("color equal", np.array_equal(a[0], b[0]), "lang equal", np.array_equal(a[1], b[1]))
for k in ("ranges", "final_T", "n_contrib", "point_list"):
    print(k, "equal", np.array_equal(a[2][k], b[2][k]))
