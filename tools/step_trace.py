"""Kernel timeline of the bench's language step, eager or as a captured graph (measurement aid):

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/st_graph -o t -- python3 tools/step_trace.py graph
    (ST_CONFIG=C5 for another BASELINE config; modes: eager, graph, pgraph; ST_BUCKET=1: pgraph with the
    N > 1 structure)
    python3 tools/step_trace.py --summary gpurun_out/st_graph/t_kernel_trace.csv

The summary prints, per step (one preprocess launch to the next), the span, the summed kernel time
and the idle gaps between consecutive kernels, so graph replay and eager launches can be compared.
"""
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(mode, steps=30):
    import torch
    import bench
    from langsplat_amd.graph import GraphedStep
    from langsplat_amd.synthetic import CONFIGS, make_cameras, make_gaussians
    c = CONFIGS[os.environ.get("ST_CONFIG", "C3")]
    P, W, H = c["P"], c["width"], c["height"]
    dev = torch.device("cuda", 0)
    params = make_gaussians(P, seed=0).to(dev)
    model = bench.Model(params, include_feature=True)
    cam = make_cameras(1, W, H, device=dev)[0]
    bg = torch.zeros(3, device=dev)
    gen = torch.Generator().manual_seed(100)
    gt = torch.nn.functional.normalize(torch.randn((3, H, W), generator=gen), dim=0).to(dev)
    mask = (torch.rand((1, H, W), generator=gen) < 0.9).to(dev)
    optim = bench.AmdAdam([{"params": [model._language_feature], "lr": 0.0025}], lr=0.0, eps=1e-15)

    def fwd_bwd():
        loss = bench.render(cam, model, bench.Pipe, bg, bench.Opt, language_target=(gt, mask))["language_l1"]
        loss.backward()
        return loss

    if mode == "graph":
        g = GraphedStep(fwd_bwd, [model._language_feature], optimizer=optim).capture()

        def step():
            g.replay()
    elif mode == "pgraph":  # the pipelined step (langsplat_amd.pipeline.PipelinedGraphStep)
        from langsplat_amd.pipeline import PipelinedGraphStep
        fwd_bwd()
        optim.step()
        optim.zero_grad(set_to_none=True)
        # ST_BUCKET=1: the N > 1 structure (a GradBucket; no process group, so its all-reduce is a no-op);
        # ST_BUCKET=rccl: the same around a one-rank RCCL group (LSR_GRAPH_COLLECTIVE=0: the collective
        # launched between the graphs, as at N > 1)
        from langsplat_amd.distributed import GradBucket
        if os.environ.get("ST_BUCKET") == "rccl":
            import torch.distributed as dist
            from langsplat_amd import launch
            dist.init_process_group("nccl", rank=0, world_size=1,
                                    init_method=f"tcp://127.0.0.1:{launch.free_port()}")
        bucket = GradBucket([model._language_feature]) if os.environ.get("ST_BUCKET") in ("1", "rccl") else None
        pg = PipelinedGraphStep(lambda: bench.render(cam, model, bench.Pipe, bg, bench.Opt,
                                                     language_target=(gt, mask))["language_l1"],
                                [model._language_feature], optim, bucket=bucket).capture()

        wait = os.environ.get("LSR_TRACE_NOWAIT", "0") != "1"

        def step():
            pg.replay(wait=wait)
    else:
        def step():
            fwd_bwd()
            optim.step()
            optim.zero_grad(set_to_none=True)
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()


def per_kernel(path):
    import collections
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        acc[r["Kernel_Name"][:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return {k: (len(v), sum(v[-20:]) / len(v[-20:])) for k, v in acc.items()}


def summary(path):
    rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path))))
    starts = [i for i, r in enumerate(rows) if "k_preprocess<" in r[2]]
    out = []
    for a, b in zip(starts[-21:-1], starts[-20:]):
        seg = rows[a:b]
        span = seg[-1][1] - seg[0][0]
        busy = sum(e - s for s, e, _ in seg)
        gaps = [(seg[i + 1][0] - seg[i][1], seg[i][2][:40], seg[i + 1][2][:40]) for i in range(len(seg) - 1)]
        out.append((span, busy, gaps))
    n = len(out)
    print(f"{n} steps: span {sum(o[0] for o in out) / n / 1e3:.1f} us, kernels {sum(o[1] for o in out) / n / 1e3:.1f} us, "
          f"kernels per step {len(out[0][2]) + 1}")
    gsum = {}
    for o in out:
        for i, (g, x, y) in enumerate(o[2]):
            gsum.setdefault(i, [0, x, y])[0] += g
    for i, (g, x, y) in sorted(gsum.items()):
        print(f"  gap {g / n / 1e3:7.2f} us  after {x}  before {y}")


def timeline(path, anchor="k_render_forward<"):
    """Kernels of the last few steps, each with its start and end relative to the step's anchor
    kernel's start (pipelined steps overlap, so kernels are listed by start time)."""
    rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path))))
    starts = [i for i, r in enumerate(rows) if anchor in r[2]]
    a, b = starts[-3], starts[-2]
    t0 = rows[a][0]
    print(f"step span (anchor to anchor): {(rows[b][0] - t0) / 1e3:.1f} us")
    for s, e, n in rows[a - 12:b + 1]:
        print(f"  {(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {n[:70]}")


if __name__ == "__main__":
    if sys.argv[1] == "--summary":
        summary(sys.argv[2])
    elif sys.argv[1] == "--timeline":
        timeline(sys.argv[2])
    elif sys.argv[1] == "--compare":  # per-kernel average (last 20 launches) of two traces
        a, b = per_kernel(sys.argv[2]), per_kernel(sys.argv[3])
        for k in sorted(set(a) | set(b), key=lambda k: -max(a.get(k, (0, 0))[1], b.get(k, (0, 0))[1])):
            print(f"{a.get(k, (0, 0))[1]:8.1f} {b.get(k, (0, 0))[1]:8.1f}  {k}")
    else:
        run(sys.argv[1])
