"""Losses of K language steps of the C3 bench view in several step forms (diagnostic aid):

    python3 tools/diag_pg.py [K]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from langsplat_amd.graph import GraphedStep
    from langsplat_amd.optim import Adam
    from langsplat_amd.pipeline import PipelinedGraphStep
    from langsplat_amd.render import render
    from langsplat_amd.synthetic import CONFIGS, make_cameras, make_gaussians
    from tests.test_gpu_fused import _Model, _Opt, _Pipe
    from tests.test_gpu_timed_step import bench_target
    os.environ["LANGSPLAT_AMD_FUSED"] = "1"
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    cfg = os.environ.get("DIAG_CFG", "C3")
    c = CONFIGS[cfg]
    P, W, H = c["P"], c["width"], c["height"]
    dev = "cuda"
    g = make_gaussians(P, seed=0)
    cam = make_cameras(1, W, H, device=dev)[0]
    gt, mask = (t.to(dev) for t in bench_target(H, W, 0))
    bg = torch.zeros(3, device=dev)

    def model():
        m = _Model(g, dev)
        for n in ("xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity"):
            getattr(m, "_" + n).requires_grad_(False)
        return m, Adam([{"params": [m._language_feature], "lr": 0.0025, "name": "l"}], lr=0.0, eps=1e-8)

    out = {}
    for run in ("eager", "eager2"):
        m, opt = model()
        ls = []
        for _ in range(K):
            loss = render(cam, m, _Pipe, bg, _Opt, language_target=(gt, mask))["language_l1"]
            loss.backward()
            opt.step()
            opt.zero_grad(set_to_none=True)
            ls.append(float(loss.item()))
        out[run] = (ls, m._language_feature.detach().clone())
    for fused in ("1", "0"):
        os.environ["LSR_FUSED_TAIL"] = fused
        m, opt = model()

        def step():
            loss = render(cam, m, _Pipe, bg, _Opt, language_target=(gt, mask))["language_l1"]
            loss.backward()
            return loss
        gs = GraphedStep(step, [m._language_feature], optimizer=opt).capture()
        ls = [float(gs.replay().item()) for _ in range(K)]
        out[f"graph fused={fused}"] = (ls, m._language_feature.detach().clone())
        for S in (2, 3):
            m, opt = model()
            pg = PipelinedGraphStep(lambda: render(cam, m, _Pipe, bg, _Opt, language_target=(gt, mask))["language_l1"],
                                    [m._language_feature], opt, sets=S).capture()
            ls = [float(pg.replay().item()) for _ in range(K)]
            pg.synchronize()
            torch.cuda.synchronize()
            out[f"pgraph S={S} fused={fused}"] = (ls, m._language_feature.detach().clone())
    ref = out["eager"][1]
    for k, (ls, p) in out.items():
        d = (p - ref).abs()
        print(f"{k:24s} " + " ".join(f"{x:.8f}" for x in ls) + f"  param max|d| {float(d.max()):.3e} "
              f"n>1e-5 {int((d > 1e-5).sum())}", flush=True)


if __name__ == "__main__":
    main()
