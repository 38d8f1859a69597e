"""bench.py -- LangSplat train step on MI355X: rasterizer fwd+bwd blends/s and train-step ms.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3|C2|C4|C5] [--no-cpu-baseline]

BASELINE.json metric: "train-step ms & Gaussian-pixel blends/sec (fwd+bwd) @1M Gaussians 1080p,
1/2/4/8 GPU".  One step mirrors train.py:76-138 in LangSplat's language-feature mode
(include_feature=True, the default of arguments/__init__.py:84): render() of one view (activations
+ the rasterizer forward, gaussian_renderer/__init__.py:19-115), masked L1 on the language image
(train.py:96-99), loss.backward(), [N>1: one RCCL all-reduce of the trainable gradient bucket],
Adam step, zero_grad.  The timed backward computes the gradients autograd asks for: in the
language step every geometry parameter is frozen (scene/gaussian_model.py:203-217), so the
rasterizer backward replays every blend but produces only dL/dmeans2D and dL/dlanguage_feature.
The same step with every geometry gradient computed as well (what the reference extension does)
is timed separately and reported beside it as `ms_per_step_all_gradients`, never as `value`; so is
the inference forward (render.py's render() under torch.no_grad(), `ms_forward_only`).

N = 1 runs BASELINE configs[2] (C3: 1M Gaussians, one 1920x1080 camera); N > 1 runs configs[3]
(C4: the same scene, camera `rank % 8` of 8 on a circle, one per GPU: weak scaling).  Data is
synthetic (seeded).  `value` = Gaussian-pixel blends (sum of n_contrib, the
forward's contributor counts = the pairs the backward replays) of all ranks per step x steps /
max-over-ranks wall time of the timed steps.
"""
from __future__ import annotations

import argparse
import gc
import json
import math
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from langsplat_amd import _native, launch, rccl  # noqa: E402
from langsplat_amd.distributed import GradBucket, collective_capturable, init_from_env  # noqa: E402
from langsplat_amd.optim import Adam as AmdAdam  # noqa: E402
from langsplat_amd.pipeline import PipelinedGraphStep, ViewPipeline  # noqa: E402
from langsplat_amd.render import render  # noqa: E402
from langsplat_amd.synthetic import CONFIGS, activated_inputs, make_cameras, make_gaussians  # noqa: E402

METRIC = "train-step ms & Gaussian-pixel blends/sec (fwd+bwd) @1M Gaussians 1080p, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip parameters (8.0 TB/s spec)


class Model:
    """GaussianModel's getters over synthetic raw parameters (scene/gaussian_model.py:134-164)."""

    def __init__(self, params, include_feature=True):
        self.max_sh_degree = params.max_sh_degree
        self.active_sh_degree = params.max_sh_degree
        self._xyz = torch.nn.Parameter(params.xyz, requires_grad=not include_feature)
        self._features_dc = torch.nn.Parameter(params.features_dc, requires_grad=not include_feature)
        self._features_rest = torch.nn.Parameter(params.features_rest, requires_grad=not include_feature)
        self._scaling = torch.nn.Parameter(params.scaling, requires_grad=not include_feature)
        self._rotation = torch.nn.Parameter(params.rotation, requires_grad=not include_feature)
        self._opacity = torch.nn.Parameter(params.opacity, requires_grad=not include_feature)
        self._language_feature = torch.nn.Parameter(params.language_feature, requires_grad=include_feature)
        # scene/gaussian_model.py:33-41 setup_functions; render() fuses these into the kernels
        self.scaling_activation = torch.exp
        self.opacity_activation = torch.sigmoid
        self.rotation_activation = torch.nn.functional.normalize

    def trainable(self):
        return [p for p in (self._xyz, self._features_dc, self._features_rest, self._opacity, self._scaling,
                            self._rotation, self._language_feature) if p.requires_grad]

    @property
    def get_xyz(self):
        return self._xyz

    @property
    def get_scaling(self):
        return torch.exp(self._scaling)

    @property
    def get_rotation(self):
        return torch.nn.functional.normalize(self._rotation)

    @property
    def get_opacity(self):
        return torch.sigmoid(self._opacity)

    @property
    def get_features(self):
        return torch.cat((self._features_dc, self._features_rest), dim=1)

    @property
    def get_language_feature(self):
        return self._language_feature

    def get_covariance(self, scaling_modifier=1.0):
        raise NotImplementedError("compute_cov3D_python is off in the benchmark (PipelineParams default)")


class Pipe:
    convert_SHs_python = False
    compute_cov3D_python = False
    debug = False


class Opt:
    include_feature = True


class OptRGB:
    """arguments/__init__.py:74-94 OptimizationParams for the RGB stage (include_feature=False)."""
    include_feature = False
    position_lr_init = 0.00016
    feature_lr = 0.0025
    opacity_lr = 0.05
    scaling_lr = 0.005
    rotation_lr = 0.001
    lambda_dssim = 0.2


def _ssim_taps(window_size, channels, device):
    """utils/loss_utils.py:24-33's 11 x 11 window (sigma 1.5) is the outer product g g^T of the 1-D
    Gaussian g: returned as its two separable factors, one per channel."""
    x = torch.arange(window_size, dtype=torch.float64) - window_size // 2
    g = torch.exp(-x * x / (2 * 1.5 ** 2))
    g = (g / g.sum()).float()
    return (g.view(1, 1, window_size, 1).expand(channels, 1, window_size, 1).contiguous().to(device),
            g.view(1, 1, 1, window_size).expand(channels, 1, 1, window_size).contiguous().to(device))


def ssim(img1, img2, window_size=11):
    """utils/loss_utils.py:35-63 (size_average=True) as torch ops: the RGB stage's loss consumer of
    the rasterizer output (outside the hot path).  The five windowed means
    (mu1, mu2, E[x1^2], E[x2^2], E[x1 x2]) are one separable pass over 15 stacked channels (an 11 x 1
    then a 1 x 11 depthwise convolution, zero padded as the 11 x 11 one: the same sums, a different
    rounding order) instead of five 11 x 11 depthwise convolutions."""
    F = torch.nn.functional
    c = img1.size(-3)
    pad = window_size // 2
    x = torch.cat([img1, img2, img1 * img1, img2 * img2, img1 * img2], dim=-3).unsqueeze(0)
    gv, gh = _ssim_taps(window_size, 5 * c, img1.device)
    m = F.conv2d(F.conv2d(x, gv.type_as(x), padding=(pad, 0), groups=5 * c), gh.type_as(x), padding=(0, pad),
                 groups=5 * c)[0]
    mu1, mu2, e11, e22, e12 = m.split(c, dim=-3)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s1, s2, s12 = e11 - mu1_sq, e22 - mu2_sq, e12 - mu1_mu2
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    r = ((2 * mu1_mu2 + C1) * (2 * s12 + C2)) / ((mu1_sq + mu2_sq + C1) * (s1 + s2 + C2))
    return r.mean()


class RGBStep:
    """The RGB stage's train step (train.py:76-138 with include_feature=False): render, the loss of
    train.py:100-103 ((1 - lambda_dssim) L1 + lambda_dssim (1 - SSIM) on the colour image), backward
    through every geometry / appearance gradient, the densification statistics of train.py:125-126
    (one kernel), Adam over the six groups of scene/gaussian_model.py:219-226 (one launch), zero_grad.
    N > 1: the six gradients and the statistics in one GradBucket all-reduce, max radii by MAX."""

    def __init__(self, params, cam, gt_image, bucket_world=1, spatial_lr_scale=1.0):
        self.model = Model(params, include_feature=False)
        self.cam, self.gt = cam, gt_image
        P = params.P
        dev = params.xyz.device
        o = OptRGB
        m = self.model
        groups = [{"params": [m._xyz], "lr": o.position_lr_init * spatial_lr_scale, "name": "xyz"},
                  {"params": [m._features_dc], "lr": o.feature_lr, "name": "f_dc"},
                  {"params": [m._features_rest], "lr": o.feature_lr / 20.0, "name": "f_rest"},
                  {"params": [m._opacity], "lr": o.opacity_lr, "name": "opacity"},
                  {"params": [m._scaling], "lr": o.scaling_lr, "name": "scaling"},
                  {"params": [m._rotation], "lr": o.rotation_lr, "name": "rotation"}]
        self.optim = AmdAdam(groups, lr=0.0, eps=1e-15)
        # scene/gaussian_model.py:196-201 training_setup state of the densification statistics
        self.max_radii2D = torch.zeros((P,), device=dev)
        self.xyz_gradient_accum = torch.zeros((P, 1), device=dev)
        self.denom = torch.zeros((P, 1), device=dev)
        self.bucket = GradBucket(m.trainable(), densify_points=P) if bucket_world > 1 else None
        self.bg = torch.zeros(3, device=dev)

    def __call__(self):
        pkg = render(self.cam, self.model, Pipe, self.bg, OptRGB)
        image = pkg["render"]
        Ll1 = torch.abs(image - self.gt).mean()
        # MIOpen has no tuned kernel for SSIM's fp32 depthwise 11 x 1 / 1 x 11 convolutions and falls
        # back to its naive ones (~9 of the 9.7 ms RGB step, profiles/r04_C3_rgb_kernel_stats.csv); ATen's
        # own depthwise kernels run them, forward and backward (LSR_SSIM_MIOPEN=1 keeps MIOpen)
        with torch.backends.cudnn.flags(enabled=os.environ.get("LSR_SSIM_MIOPEN", "0") == "1"):
            loss = (1.0 - OptRGB.lambda_dssim) * Ll1 + OptRGB.lambda_dssim * (1.0 - ssim(image, self.gt))
            loss.backward()
        vgrad = pkg["viewspace_points"].grad
        if self.bucket is None:
            _native.densification_stats(pkg["radii"], vgrad, self.max_radii2D, self.xyz_gradient_accum, self.denom)
            self.optim.step()
            self.optim.zero_grad(set_to_none=True)
        else:
            self.bucket.stage_densification(pkg["radii"], vgrad, self.max_radii2D)
            self.bucket.all_reduce(average=True)
            self.bucket.apply_densification(self.xyz_gradient_accum, self.denom)
            self.optim.step()
            self.bucket.zero()
        return loss


def algorithmic_bytes(stage, P, V, R, HW, M, color_grad=True, geometry=True, fused_loss=False):
    """Compulsory HBM bytes per launch of each stage (SURVEY.md §8d per-unit model).
    The render backward's per-pixel and per-Gaussian terms follow its variant: dL/dcolor is read
    only when the colour image reaches the loss, and the per-Gaussian record it accumulates holds
    12 values with geometry gradients, 5 (dmean2D x/y + language) without.  fused_loss: the forward
    also reads the target (12 B/px) and mask (1) and writes a 1-B sign code, which the backward
    reads instead of dL/dlanguage (12 B/px)."""
    sh = 12 * M
    bwd_px = 4 + 4 + (1 if fused_loss else 12) + (12 if color_grad else 0)  # T, count, dL/dlang | code, [dL/dcolor]
    fwd_px = 32 + (14 if fused_loss else 0)
    bwd_g = 4 * (12 if geometry else 5)
    return {
        # reads means 12, scale 12, rot 16, opacity 4, SH, lang 12; writes radii 4 + key 4 + tiles 4
        # + rect 8 + clamp 4 (all P) and the 48 B record for visible Gaussians
        "preprocess": P * (12 + 12 + 16 + 4 + sh + 12 + 24) + V * 48,
        # per instance: list id 4 + gathered record 48; per pixel: colour 12 + language 12 + T 4 + count 4
        "render forward": R * 52 + HW * fwd_px,
        # per instance: id 4 + record 48; per pixel: bwd_px; per visible Gaussian: its gradient
        # record, accumulated once
        "render backward": R * 52 + HW * bwd_px + V * bwd_g,
        # reads means/scale/rot/SH/radii/clamp + 48 B grad record; writes every gradient output
        "preprocess backward": P * (12 + 12 + 16 + sh + 4 + 4) + V * 48 + P * (12 + 12 + 12 + 4 + 12 + sh + 12 + 16),
    }.get(stage)


def survey_step_bytes(P, R, HW, M, geometry):
    """SURVEY.md §8d's implementation-independent traffic model of one rasterizer fwd+bwd,
    bytes = P*B_G + I*B_I + HW*B_px, with B_G following the gradients the step computes: with
    geometry gradients 312 + 36M (§8d as written); in the language step (geometry frozen) the
    preprocess backward's reads (76 + 12M) and writes (40 + 12M) are replaced by what the
    gradient epilogue moves (the 5-value record 20 in, dL/dmeans2D 12 + dL/dlanguage 12 out) and
    the render backward's record is 5 values (2 x 20) instead of 12 (2 x 48); the language
    feature's own read (12) is added in both.  B_I = 148, B_px = 64 (§8d)."""
    sh = 12 * M
    if geometry:
        b_g = 312 + 3 * sh + 12
    else:
        b_g = (44 + sh) + 48 + 8 + 2 * 20 + (20 + 24) + 12
    return P * b_g + R * 148 + HW * 64


def compulsory_bytes(stage, P, V, R, HW, M, **variant):
    """The compulsory-bytes form of algorithmic_bytes: a render kernel reads each
    visible Gaussian's 48-B record from HBM once -- its re-reads for the other tiles it touches are
    L2 / MALL hits -- and of an instance only its 4-B list id; per pixel and per Gaussian as there.
    The other stages stream their operands once already: the same bytes."""
    lit = algorithmic_bytes(stage, P, V, R, HW, M, **variant)
    if lit is None or stage not in ("render forward", "render backward"):
        return lit
    return lit - R * 52 + R * 4 + V * 48


def compulsory_step_bytes(P, V, R, HW, M, geometry):
    """survey_step_bytes with the compulsory per-instance and per-record terms: B_I = 12 (the list id
    written once, read by the forward and the backward) instead of 148, plus each visible Gaussian's
    48-B record read once by each render kernel (the 2 x 52 B of §8d's per-instance gathers)."""
    return survey_step_bytes(P, R, HW, M, geometry) - R * 148 + R * 12 + V * 96


def hbm_view(nbytes, seconds, model):
    """A bytes / time rate against the HBM peak.  A fraction above 1 is not reported (VERDICT r05 item
    4b): no kernel moves more than the peak, so such a model counts bytes that never reach HBM (re-reads
    served by L2 / MALL); `frac` is then null and `frac_refused` names the model."""
    ach = nbytes / seconds / 1e9
    f = ach / HBM_PEAK_GBS
    out = {"bound": "hbm", "model": model, "bytes": int(nbytes), "achieved": round(ach, 2), "peak": HBM_PEAK_GBS,
           "unit": "GB/s", "frac": round(f, 4) if f <= 1.0 else None}
    if f > 1.0:
        out["frac_refused"] = (f"{model}: {f:.3f} x peak -- more bytes than HBM can move in the measured time, "
                               "so the model counts re-reads that L2 / MALL serve")
    return out


# the stage that dominates the step (measured: profiles/r02_summary.json); timed live in the bench
DOMINANT_STAGE = "render backward"

# rocprofv3 names of the bench step's kernels (template arguments: k_render_forward<kStats, kFeat, kLoss>,
# k_render_backward<kStats, kFeat, kColor, kGeo>; the language step runs kColor = kGeo = false)
STAGE_KERNEL = {"render backward": "lsr::k_render_backward<false, true, false, false>",
                "render forward": "lsr::k_render_forward<false, true, true>",
                "preprocess": "lsr::k_preprocess<2>", "preprocess backward": "lsr::k_preprocess_backward"}


# profiles this round's bench reads its PMC figures from: profiles/<ROUND>_<config>_{summary,valu}.json
# (tools/profile_round.sh + tools/prof_summary.py, tools/pmc_valu.sh + tools/valu_summary.py).  A
# profile of another round or another config is never used: its field is then null.
ROUND = "r06"
CUS = 256
CLOCK_HZ = 2.4e9  # MI355X_MICROARCH.md: max engine clock (what the PMC runs' GRBM_GUI_ACTIVE / time gives)
# wave64 VALU instructions a CU can issue per cycle: 4 SIMD-32 units, each one wave64 instruction per
# 2 cycles when two or more waves alternate (MI355X_MICROARCH.md "Wave scheduling"; tools/valu_peak.hip
# measures it: profiles/r03_valu_peak.txt)
VALU_PEAK_PER_CU_CYCLE = 2.0


def _profile(kind, cfg):
    path = os.path.join(ROOT, "profiles", f"{ROUND}_{cfg}_{kind}.json")
    try:
        return json.load(open(path))["kernels"], os.path.relpath(path, ROOT)
    except (OSError, ValueError, KeyError):
        return None, None


def pmc_traffic(stage, cfg):
    """HBM bytes per launch of the stage's kernel from this round's PMC summary of this config
    (FETCH_SIZE + WRITE_SIZE passes, gfx950 correction: tools/prof_summary.py), or (None, None)."""
    k, src = _profile("summary", cfg)
    d = (k or {}).get(STAGE_KERNEL.get(stage), {})
    return (float(d["hbm_bytes_per_launch"]), src) if "hbm_bytes_per_launch" in d else (None, None)


def pmc_valu(stage, cfg):
    """SQ_INSTS_VALU per launch of the stage's kernel (and the PMC run's own per-CU-cycle rate) from
    this round's profiles/<ROUND>_<cfg>_valu.json (tools/valu_summary.py), or (None, None, None)."""
    k, src = _profile("valu", cfg)
    d = (k or {}).get(STAGE_KERNEL.get(stage), {})
    if d.get("valu_insts") is None:
        return None, None, None
    return float(d["valu_insts"]), d.get("valu_per_cu_cycle"), src


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(cfg, seconds_budget=25.0):
    """The C oracle (oracle/lsr_oracle.c, OpenMP over tiles on all the threads OMP_NUM_THREADS grants)
    on the FULL workload config: the same scene, camera and resolution, one forward + full backward
    (every gradient) per run, runs repeated while within the budget (at most 3), median rate."""
    from oracle import oracle
    from tests.scenes import settings_for
    c = CONFIGS[cfg]
    g = make_gaussians(c["P"], seed=0)
    cam = make_cameras(c["views"], c["width"], c["height"])[0]
    st = settings_for(cam, sh_degree=3)
    with torch.no_grad():
        inp = {k: v.contiguous() for k, v in activated_inputs(g).items()}
    H, W = c["height"], c["width"]
    gen = torch.Generator().manual_seed(1)
    gcol = torch.randn((3, H, W), generator=gen) / (3 * H * W)
    glang = torch.randn((3, H, W), generator=gen) / (3 * H * W)
    times, blends = [], 0
    t_start = time.perf_counter()
    while len(times) < 3 and (not times or time.perf_counter() - t_start + times[-1] < seconds_budget):
        t0 = time.perf_counter()
        run = oracle.forward(st, **inp)
        run.backward(gcol, glang)
        times.append(time.perf_counter() - t0)
        blends = run.blends
        del run
    dt = sorted(times)[len(times) // 2]
    threads = oracle.num_threads()
    return {"value": round(blends / dt, 1), "unit": "blends/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(),
            "sample": f"{cfg} full scene ({c['P']} Gaussians, {W}x{H}, camera 0), forward + full backward "
                      f"(every gradient), {blends} blends, median of {len(times)} run(s) "
                      f"({', '.join(f'{t:.2f}' for t in times)} s), C oracle on {threads} OpenMP threads"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)  # ~70 ms timed: averages out host jitter
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--json-out", default=None)
    args = ap.parse_args()
    if launch.should_launch(args.gpus):
        # a plain `python bench.py --gpus N`: start the N ranks here (before anything touches the GPU)
        sys.exit(launch.launch([os.path.abspath(__file__)] + sys.argv[1:], args.gpus))

    rank, world = init_from_env()
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the process group has {world} rank(s)")
    backend = dist.get_backend() if world > 1 else None
    if backend == "nccl" and world > torch.cuda.device_count():
        raise SystemExit(f"bench.py: {world} RCCL ranks need {world} GPUs ({torch.cuda.device_count()} visible); "
                         "LSR_DIST_BACKEND=gloo rehearses several ranks on one GPU")
    # one GPU per rank; the modulo only matters for a gloo rehearsal of N ranks on fewer GPUs
    local_rank = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    cfg = args.config or ("C3" if world == 1 else "C4")
    c = CONFIGS[cfg]
    P, W, H = c["P"], c["width"], c["height"]
    view = rank % c["views"] if c["views"] > 1 else 0

    params = make_gaussians(P, seed=0, sh_degree=c["sh_degree"]).to(dev)
    model = Model(params, include_feature=True)
    cam = make_cameras(c["views"], W, H, device=dev)[view]
    bg = torch.zeros(3, device=dev)
    gen = torch.Generator().manual_seed(100 + view)
    gt = torch.nn.functional.normalize(torch.randn((3, H, W), generator=gen), dim=0).to(dev)
    # scene/cameras.py:72 builds the mask as a bool tensor (seg != -1)
    mask = (torch.rand((1, H, W), generator=gen) < 0.9).to(dev)
    fused = os.environ.get("LANGSPLAT_AMD_FUSED", "1") != "0"
    # scene/gaussian_model.py:229 Adam(lr=0.0, eps=1e-15) over the language-feature group (:203-217)
    groups = [{"params": [model._language_feature], "lr": 0.0025, "name": "language_feature"}]
    if fused:  # one HIP kernel per parameter
        optim = AmdAdam(groups, lr=0.0, eps=1e-15)
    else:
        optim = torch.optim.Adam(groups, lr=0.0, eps=1e-15, fused=True)
    # N > 1: .grad tensors are views of one flat bucket (one all-reduce); N = 1: train.py:138's
    # zero_grad(set_to_none=True), so autograd hands the rasterizer's gradient over without a copy
    # (LSR_BENCH_BUCKET=1 at N = 1: the N > 1 step structure around a one-rank RCCL all-reduce -- a
    # measurement aid for the cost of the N > 1 form itself, collective eager between two graphs or,
    # with LSR_GRAPH_COLLECTIVE=1, captured; LSR_BENCH_BUCKET=nodist: no process group, no collective)
    bench_bucket = os.environ.get("LSR_BENCH_BUCKET", "0")
    if world == 1 and bench_bucket == "1" and not dist.is_initialized():
        dist.init_process_group("nccl", rank=0, world_size=1,
                                init_method=f"tcp://127.0.0.1:{launch.free_port()}")
    bucket = GradBucket(model.trainable()) if world > 1 or bench_bucket in ("1", "nodist") else None

    def step():
        if fused:  # the loss inside the compositing kernel, its backward in the replay
            loss = render(cam, model, Pipe, bg, Opt, language_target=(gt, mask))["language_l1"]
        else:      # train.py:98 + utils/loss_utils.py:17-18 as torch ops
            lang = render(cam, model, Pipe, bg, Opt)["language_feature_image"]
            loss = torch.abs(lang * mask - gt * mask).mean()
        loss.backward()
        if bucket is not None:
            bucket.all_reduce(average=True)
        optim.step()
        optim.zero_grad(set_to_none=bucket is None or bucket.direct)
        return loss

    # blends and instance counts of this view (constant over steps: geometry is frozen)
    with torch.no_grad():
        inp = activated_inputs(params)
        from langsplat_amd.render import GaussianRasterizationSettings
        st = GaussianRasterizationSettings(H, W, math.tan(cam.FoVx * 0.5), math.tan(cam.FoVy * 0.5), bg, 1.0,
                                           cam.world_view_transform, cam.full_proj_transform, 3,
                                           cam.camera_center, False, False, True)
        nr, _, _, radii, geom, binning, image = _native.rasterize_gaussians(
            st, inp["means3D"], inp["shs"], None, inp["language_feature_precomp"], inp["opacities"],
            inp["scales"], inp["rotations"], None)
        lay = _native.state_layout(P, W, H, nr)
        ncon = image[lay["n_contrib"]:lay["n_contrib"] + 4 * W * H].view(torch.int32)
        blends = int(ncon.to(torch.int64).sum().item())
        visible = int((radii > 0).sum().item())
        del geom, binning, image, inp

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # the collector stays off inside the timed loops (as timeit does): a collection of the steps'
    # autograd garbage would land on the host's critical path of one step
    gc.collect()
    gc.disable()

    # eager passes first (the captured graph then owns the parameters' .grad tensors):
    # (2) the same step with every geometry gradient computed although no parameter needs one (what
    # the reference extension does; LSR_ALL_GRADS=1): reported beside, never as `value`
    _native.FORCE_GEOMETRY_GRADS = True
    for _ in range(2):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed_all = time.perf_counter() - t1
    _native.FORCE_GEOMETRY_GRADS = os.environ.get("LSR_ALL_GRADS", "0") == "1"
    # (2b) the inference form (render.py:24-55: render() under torch.no_grad(), LSR_FWD_NO_BACKWARD):
    # the forward alone, reported beside, never as `value`
    with torch.no_grad():
        for _ in range(2):
            render(cam, model, Pipe, bg, Opt)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            render(cam, model, Pipe, bg, Opt)
        torch.cuda.synchronize()
        elapsed_fwd = time.perf_counter() - t1
    # (3) the eager step itself (the host enqueues every launch, one wait per forward)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    te = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed_eager = time.perf_counter() - te
    # (3b) the dominant kernel's average launch time, HIP events around it on its stream (every step)
    _native.profile_enable(True, stages=[DOMINANT_STAGE], every=1)
    for _ in range(min(args.steps, 20)):
        step()
    torch.cuda.synchronize()
    _native.profile_enable(False)
    dom = _native.profile_report().get(DOMINANT_STAGE, {"avg_ms": float("nan")})
    # (4) stage breakdown: every stage profiled
    prof_steps = min(args.steps, 10)
    _native.profile_enable(True)
    for _ in range(prof_steps):
        step()
    torch.cuda.synchronize()
    _native.profile_enable(False)
    prof = _native.profile_report()

    # (5) the pipelined form (langsplat_amd.pipeline.ViewPipeline): consecutive steps on two alternating
    # streams, each forward deferring the language feature until the previous update has landed, so the
    # next view's geometry stages run beside this view's backward, [all-reduce] and Adam.  Eager launches.
    elapsed_pipe = float("inf")
    if fused and os.environ.get("LSR_PIPELINE", "1") != "0":
        pipe = ViewPipeline(optim, bucket=bucket)
        optim.zero_grad(set_to_none=True)

        def run_pipe():
            with pipe.step():
                loss = render(cam, model, Pipe, bg, Opt, language_target=(gt, mask))["language_l1"]
                loss.backward()
                pipe.update()
            return loss
        for _ in range(3):
            run_pipe()
        pipe.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        tp = time.perf_counter()
        for _ in range(args.steps):
            run_pipe()
        pipe.synchronize()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed_pipe = time.perf_counter() - tp
        del pipe

    # The serial HIP-graph form (langsplat_amd.graph.GraphedStep: the whole step as one graph per
    # replay) is not timed here: its kernels sum to the eager step's (502.6 vs 498.8 us under the
    # kernel tracer, profiles/r05_graph_vs_eager.txt), and each replay adds a graph boundary (idle
    # queue between consecutive graph launches) that the eager launches do not pay
    # (driver, round 4: 0.521 vs 0.497 ms).  The pipelined graph below is the captured form.
    graphed = fused and os.environ.get("LSR_GRAPH", "1") != "0"
    # (6) the pipelined order as HIP graphs on two streams (langsplat_amd.pipeline.PipelinedGraphStep):
    # each replay is one full step -- this view's compositing, loss, backward and Adam on one stream, the
    # next view's geometry stages (the forward's first half) on the other -- with no host work inside
    elapsed_pg = elapsed_sync = float("inf")
    pg_rot = None
    pg_reps = []

    def run_pipelined_graph():
        """The pipelined graph form's timed steps, reps and with-sync steps."""
        reps = []
        # N > 1: the bucket's all-reduce (RCCL) is launched between each set's backward and Adam graphs
        # rotation (N = 1): R steps per stream-A graph (pipeline.py), R dividing the timed steps
        rot = 1
        if bucket is None:
            want = int(os.environ.get("LSR_PG_ROT", "1"))
            rot = max(r for r in range(1, want + 1) if args.steps % r == 0)
        pg = PipelinedGraphStep(lambda: render(cam, model, Pipe, bg, Opt, language_target=(gt, mask))["language_l1"],
                                model.trainable(), optim, bucket=bucket, rotation=rot, model=model)
        pg.capture()
        # untimed replays until the two streams' steady state: the first replays after a capture run
        # slower (profiles/r05_bench_first.json: timed steps 0.4115 ms after 20 warm replays, its reps
        # 0.399), and a timed pass that starts before the streams have settled can stay at the slow
        # level (a run with 20: 0.4467 timed, reps 0.4032-0.4039): 200 replays (~80 ms at C3)
        warm = rot * max(1, max(200, 2 * args.warmup) // rot)
        for _ in range(warm):
            pg.replay()
        torch.cuda.synchronize()
        if not pg.check():
            for _ in range(warm):
                pg.replay()
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        tq = time.perf_counter()
        # (replay(wait=False), no per-step join with the caller's stream, measured slower: 0.477 vs
        # 0.420 ms per step, tools/pg_host.py --nowait)
        for _ in range(args.steps):
            pg.replay()
        pg.synchronize()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed_pg = time.perf_counter() - tq
        if not pg.check():
            raise RuntimeError("a pipelined view exceeded its capacities during the timed steps")
        # the spread of this form over further reps of the same K steps (not `value`: the run-to-run
        # levels of DESIGN.md §5b), and train.py:108's loss.item() after every step
        # (ms_per_step_with_sync: a device-to-host sync per step, no run-ahead)
        for _ in range(int(os.environ.get("LSR_BENCH_REPS", "4"))):
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            tr = time.perf_counter()
            for _ in range(args.steps):
                pg.replay()
            pg.synchronize()
            torch.cuda.synchronize()
            reps.append(1000.0 * (time.perf_counter() - tr) / args.steps)
        for _ in range(10):  # untimed: the synced form's own warm-up (its first replays take the Python path)
            pg.replay().item()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        ts = time.perf_counter()
        for _ in range(args.steps):
            pg.replay().item()
        torch.cuda.synchronize()
        elapsed_sync = time.perf_counter() - ts
        if not pg.check():
            raise RuntimeError("a pipelined view exceeded its capacities during the timed steps")
        del pg
        return elapsed_pg, elapsed_sync, rot, reps

    pg_error = None
    if graphed and os.environ.get("LSR_PIPELINE", "1") != "0":
        if world == 1:
            elapsed_pg, elapsed_sync, pg_rot, pg_reps = run_pipelined_graph()
        else:
            # N > 1 with RCCL the collective is captured inside the step graphs, a path a one-GPU box
            # cannot run with two ranks (RCCL refuses two ranks on one GPU, profiles/r06_rccl_two_ranks_one_gpu.txt):
            # a failure there (every rank fails alike: the same capture) leaves the eager forms as `value`
            try:
                elapsed_pg, elapsed_sync, pg_rot, pg_reps = run_pipelined_graph()
            except RuntimeError as e:
                pg_error = f"{type(e).__name__}: {e}"[:400]
                print(f"rank {rank}: pipelined graph form failed: {pg_error}", file=sys.stderr, flush=True)
                torch.cuda.synchronize()
                dist.barrier()
    gc.enable()
    # the RGB stage's step on the same scene and view (all six groups trainable, L1 + SSIM, densification
    # statistics): reported beside, never as `value`
    rgb_ms = None
    if os.environ.get("LSR_BENCH_RGB", "1") != "0":
        gtimg = torch.rand((3, H, W), generator=torch.Generator().manual_seed(200 + view)).to(dev)
        rgb = RGBStep(make_gaussians(P, seed=0, sh_degree=c["sh_degree"]).to(dev), cam, gtimg, bucket_world=world)
        for _ in range(3):
            rgb()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        rgb_steps = max(1, args.steps // 2)
        for _ in range(rgb_steps):
            rgb()
        torch.cuda.synchronize()
        rgb_ms = 1000.0 * (time.perf_counter() - t2) / rgb_steps
        del rgb

    # `value`: the fastest of the full-step forms timed above (each does the whole step's work; the
    # others are reported beside it)
    forms = {"eager": elapsed_eager, "pipelined": elapsed_pipe, "pipelined_graph": elapsed_pg}
    names = sorted(forms)
    t = torch.tensor([min(forms[n], 1e30) for n in names] + [float(blends)], dtype=torch.float64, device=dev)
    if world > 1:
        tmax = t[:-1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = t[-1:].clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        times, blends_all = dict(zip(names, tmax.tolist())), float(tsum.item())
    else:
        times, blends_all = dict(zip(names, t[:-1].tolist())), float(blends)
    best = min(names, key=lambda n: times[n])
    elapsed_max = times[best]

    if rank != 0:
        dist.barrier()
        torch.cuda.synchronize()
        rccl.destroy_default()
        dist.destroy_process_group()
        return

    ms_per_step = 1000.0 * elapsed_max / args.steps
    value = blends_all * args.steps / elapsed_max
    raster_ms = sum(v["total_ms"] for k, v in prof.items()) / prof_steps
    dom_name = DOMINANT_STAGE
    M = (c["sh_degree"] + 1) ** 2
    # the language step: the colour image does not reach the loss; geometry gradients as needed
    geometry = bool(_native.FORCE_GEOMETRY_GRADS)
    variant = dict(color_grad=False, geometry=geometry, fused_loss=fused)
    bytes_dom = algorithmic_bytes(dom_name, P, visible, nr, W * H, M, **variant)
    roofline = None
    if bytes_dom is not None:
        avg_s = dom["avg_ms"] * 1e-3
        # HBM views of the dominant kernel: SURVEY.md §8d's per-unit bytes as written
        # ("literal": a Gaussian's record counted for every tile it touches) and the compulsory bytes
        # (each record once), over the live launch time; and the HBM bytes this round's PMC passes of
        # this config measured for the same kernel
        traffic, tsrc = pmc_traffic(dom_name, cfg)
        hbm = hbm_view(bytes_dom, avg_s, "SURVEY.md §8d per-launch bytes (literal)")
        hbm.update(traffic=None if traffic is None else int(traffic), traffic_source=tsrc,
                   traffic_frac=None if traffic is None else round(traffic / avg_s / 1e9 / HBM_PEAK_GBS, 4))
        hbm_c = hbm_view(compulsory_bytes(dom_name, P, visible, nr, W * H, M, **variant), avg_s,
                         "compulsory bytes (each record once, 4 B per instance)")
        # what bounds the render kernels is instruction issue, not HBM: the headline is
        # the VALU issue rate, SQ_INSTS_VALU per launch (this round's PMC pass of this config) over the
        # live launch time, against the chip's wave64 VALU issue peak
        insts, pmc_rate, vsrc = pmc_valu(dom_name, cfg)
        if insts is not None:
            achieved = insts / CUS / (avg_s * CLOCK_HZ)
            roofline = {"bound": "valu", "kernel": dom_name, "achieved": round(achieved, 4),
                        "peak": VALU_PEAK_PER_CU_CYCLE, "unit": "wave64 VALU instructions / CU / cycle",
                        "frac": round(achieved / VALU_PEAK_PER_CU_CYCLE, 4), "traffic": hbm["traffic"],
                        "avg_ms": round(dom["avg_ms"], 4), "valu_insts_per_launch": int(insts),
                        "valu_source": vsrc, "pmc_run_valu_per_cu_cycle": pmc_rate, "hbm": hbm,
                        "hbm_compulsory": hbm_c}
        else:  # no VALU profile of this round and config: the compulsory HBM view is the headline
            roofline = dict(hbm_c, kernel=dom_name, avg_ms=round(dom["avg_ms"], 4), traffic=hbm["traffic"],
                            valu_source=None, hbm=hbm, hbm_compulsory=hbm_c)
        # north_star's "% of HBM roofline" (DESIGN.md §4): the whole rasterizer fwd+bwd (every profiled
        # stage except the optimizer) against SURVEY.md §8d's step model as written, and against its
        # compulsory form; each also over the benched step (the stages overlap across two streams
        # there, and the step holds the optimizer: the rate the whole job sustains)
        raster_stage_ms = sum(v["total_ms"] for k, v in prof.items() if k != "adam") / prof_steps
        for key, sb, model in (("fwd_bwd_model", survey_step_bytes(P, nr, W * H, M, geometry),
                                "SURVEY.md §8d (literal)"),
                               ("fwd_bwd_compulsory", compulsory_step_bytes(P, visible, nr, W * H, M, geometry),
                                "SURVEY.md §8d, compulsory per-instance / per-record terms")):
            v = hbm_view(sb, raster_stage_ms * 1e-3, model)
            v["ms"] = round(raster_stage_ms, 4)
            st = hbm_view(sb, ms_per_step * 1e-3, model)
            v["step"] = {k: st[k] for k in ("achieved", "frac", "frac_refused") if k in st}
            v["step"]["ms"] = round(ms_per_step, 4)
            roofline[key] = v
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg)
        # the like-for-like GPU figure: the oracle times a forward + FULL backward (every gradient),
        # which is the step of ms_per_step_all_gradients, not the language step of `value`
        cpu["pairs_with"] = {"gpu_form": "ms_per_step_all_gradients",
                             "gpu_value": round(blends_all * args.steps / elapsed_all, 1),
                             "gpu_over_cpu": round(blends_all * args.steps / elapsed_all / cpu["value"], 1)}
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "blends/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (seeded random Gaussians / cameras, SURVEY.md §8d)",
        "config": {"workload": f"{cfg}: {P} Gaussians, {W}x{H}, SH deg 3 + 3-ch language feature, "
                               f"include_feature train step, 1 view per GPU",
                   "gaussians": P, "width": W, "height": H, "views": world, "parallelism": f"dp{world} (views)",
                   "ranks": world, "backend": backend or "none (1 rank)",
                   "blends_per_step": blends_all, "num_rendered_rank0": nr, "visible_rank0": visible,
                   "activation_and_loss": "fused" if fused else "torch",
                   "gradients": "all geometry" if _native.FORCE_GEOMETRY_GRADS else
                                "as needed: means2D + language feature (geometry frozen, "
                                "scene/gaussian_model.py:203-217)"},
        "ms_per_step_with_sync": round(1000.0 * elapsed_sync / args.steps, 4) if elapsed_sync < 1e29 else None,
        "pipelined_graph_reps_ms": {"reps": [round(x, 4) for x in pg_reps],
                                    "median": round(float(np.median(pg_reps)), 4) if pg_reps else None,
                                    "min": round(min(pg_reps), 4) if pg_reps else None,
                                    "max": round(max(pg_reps), 4) if pg_reps else None},
        "ms_per_step_eager": round(1000.0 * elapsed_eager / args.steps, 4),
        "step_form": {"eager": "eager launches, one stream",
                      "pipelined": "eager launches, consecutive views on two streams (the next view's geometry "
                                   "beside this view's backward" + (", RCCL all-reduce" if world > 1 else "")
                                   + " and Adam)",
                      "pipelined_graph": "HIP graphs on two streams: this view's compositing + loss, backward, "
                                         + ((f"{backend} all-reduce of the language partials and skip flag ("
                                             + ("in the graph" if collective_capturable() else "between two graphs")
                                             + ("; RCCL on the step's stream" if rccl.direct_enabled() else "")
                                             + "), ") if world > 1 and os.environ.get("LSR_PG_DEFER", "1") != "0"
                                            else (f"{backend} all-reduce ("
                                                  + ("in the graph" if collective_capturable() else "between two graphs")
                                                  + "), ") if world > 1 else "") +
                                         "gradient + Adam + next records' fill pass on one, the next view's "
                                         "geometry (forward split in two calls) on the other"}[best],
        "pipelined_graph_rotation": pg_rot,
        "pipelined_graph_error": pg_error,
        "ms_per_step_forms": {n: (round(1000.0 * v / args.steps, 4) if v < 1e29 else None) for n, v in times.items()},
        "ms_per_step_all_gradients": round(1000.0 * elapsed_all / args.steps, 4),
        "ms_forward_only": round(1000.0 * elapsed_fwd / args.steps, 4),
        "ms_per_step_rgb": None if rgb_ms is None else round(rgb_ms, 4),
        "raster_ms_per_step": round(raster_ms, 4),
        "stages_ms_per_step": {k: round(v["total_ms"] / prof_steps, 4) for k, v in sorted(prof.items())},
        "roofline": roofline,
        "cpu_baseline": cpu,
    }
    line = json.dumps(out)
    print(line, flush=True)
    if args.json_out:
        with open(args.json_out, "w") as f:
            f.write(line + "\n")
    if world > 1:
        dist.barrier()
    if dist.is_initialized():
        torch.cuda.synchronize()
        rccl.destroy_default()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
