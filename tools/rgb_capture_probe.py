"""Captures the RGB-stage step (render + L1 + backward through every gradient + 6-group Adam) into a
langsplat_amd.graph.GraphedStep at a given size and replays it once (diagnostic aid):

    python3 tools/rgb_capture_probe.py P W H [adam|noadam] [keepgraph]

keepgraph: an eager step's autograd graph stays alive (its output held) across the capture.
"""
import faulthandler
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
faulthandler.enable()


def main():
    import torch
    from langsplat_amd.graph import GraphedStep
    from langsplat_amd.render import render
    from langsplat_amd.synthetic import make_cameras, make_gaussians
    from tests.test_gpu_densify import _OptRGB, _rgb_model, _l1_step
    from tests.test_gpu_fused import _Pipe
    P, W, H = (int(a) for a in sys.argv[1:4])
    with_adam = (sys.argv[4] if len(sys.argv) > 4 else "adam") == "adam"
    os.environ["LANGSPLAT_AMD_FUSED"] = "1"
    dev = "cuda"
    g = make_gaussians(P, seed=0)
    cam = make_cameras(1, W, H, device=dev)[0]
    gt = torch.rand((3, H, W), generator=torch.Generator().manual_seed(1)).to(dev)
    m, opt = _rgb_model(g)
    _l1_step(m, opt, cam, gt)
    keep = None
    if "keepgraph" in sys.argv:
        keep = render(cam, m, _Pipe, torch.zeros(3, device=dev), _OptRGB)
        (keep["render"] * 1.0).sum().backward(retain_graph=True)
        opt.zero_grad(set_to_none=True)
    bg = torch.zeros(3, device=dev)
    params = [g_["params"][0] for g_ in opt.param_groups]

    def step():
        pkg = render(cam, m, _Pipe, bg, _OptRGB)
        loss = torch.abs(pkg["render"] - gt).mean()
        loss.backward()
        return loss
    print("capturing", P, W, H, "adam" if with_adam else "no adam", flush=True)
    gs = GraphedStep(step, params, optimizer=opt if with_adam else None).capture()
    print("captured", flush=True)
    loss = gs.replay()
    torch.cuda.synchronize()
    print("replayed", float(loss.item()), gs.check(), flush=True)


if __name__ == "__main__":
    main()
