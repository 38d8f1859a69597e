"""Where the pipelined step's two speed levels come from (measurement aid):

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bm -o t -- python3 tools/bimodal_trace.py run
    python3 tools/bimodal_trace.py --analyze gpurun_out/bm/t_kernel_trace.csv

`run` is tools/pg_host.py's loop (bench.py's PipelinedGraphStep at C3) with REPS reps of STEPS replays,
each rep drained and followed by a 50 ms pause, so the trace splits into reps.  `--analyze` splits the
kernel trace at those pauses, takes each rep's step time (span / steps), sorts the reps into a fast
and a slow half, and diffs them kernel by kernel (average duration, launches) and queue by queue
(busy fraction, idle gaps between consecutive kernels of the same queue).
"""
import collections
import csv
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run():
    import torch
    import bench
    from langsplat_amd.pipeline import PipelinedGraphStep
    from langsplat_amd.synthetic import CONFIGS, make_cameras, make_gaussians
    steps = int(os.environ.get("BM_STEPS", "150"))
    reps = int(os.environ.get("BM_REPS", "12"))
    c = CONFIGS["C3"]
    P, W, H = c["P"], c["width"], c["height"]
    dev = torch.device("cuda", 0)
    model = bench.Model(make_gaussians(P, seed=0).to(dev), include_feature=True)
    cam = make_cameras(1, W, H, device=dev)[0]
    bg = torch.zeros(3, device=dev)
    gen = torch.Generator().manual_seed(100)
    gt = torch.nn.functional.normalize(torch.randn((3, H, W), generator=gen), dim=0).to(dev)
    mask = (torch.rand((1, H, W), generator=gen) < 0.9).to(dev)
    optim = bench.AmdAdam([{"params": [model._language_feature], "lr": 0.0025, "name": "language_feature"}],
                          lr=0.0, eps=1e-15)
    pg = PipelinedGraphStep(lambda: bench.render(cam, model, bench.Pipe, bg, bench.Opt,
                                                 language_target=(gt, mask))["language_l1"],
                            [model._language_feature], optim, model=model).capture()
    for _ in range(20):
        pg.replay()
    pg.synchronize()
    torch.cuda.synchronize()
    for rep in range(reps):
        time.sleep(0.05)
        t0 = time.perf_counter()
        for _ in range(steps):
            pg.replay()
        pg.synchronize()
        torch.cuda.synchronize()
        print(f"rep {rep}: {1e3 * (time.perf_counter() - t0) / steps:.4f} ms/step (wall)", flush=True)


def _short(name):
    if "lsr::" in name:
        name = name[name.find("k_"):]
        return name[:name.find("(")] if "(" in name else name
    return name[:40]


def analyze(path, steps=None):
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), _short(r["Kernel_Name"]), r["Queue_Id"])
                  for r in csv.DictReader(open(path)))
    # reps: separated by pauses of > 20 ms with no kernel
    reps, cur = [], [rows[0]]
    for r in rows[1:]:
        if r[0] - max(x[1] for x in cur[-50:]) > 20_000_000:
            reps.append(cur)
            cur = []
        cur.append(r)
    reps.append(cur)
    reps = [r for r in reps if sum("k_render_forward" in x[2] for x in r) > 20]
    out = []
    for rep in reps:
        n = sum("k_render_forward" in x[2] for x in rep)
        span = (rep[-1][1] - rep[0][0]) / 1e3
        out.append((span / n, n, rep))
    print(f"{len(out)} reps: " + " ".join(f"{o[0]:.1f}" for o in out) + " us/step")
    med = statistics.median(o[0] for o in out)
    fast = [o for o in out if o[0] <= med]
    slow = [o for o in out if o[0] > med]
    if not slow:
        print("no slow reps")
        return

    def kstats(group):
        acc = collections.defaultdict(list)
        for _, _, rep in group:
            for s, e, k, q in rep[len(rep) // 10:]:  # past the rep's ramp
                acc[k].append((e - s) / 1e3)
        return acc

    kf, ks = kstats(fast), kstats(slow)
    nf = sum(o[1] for o in fast) * 0.9
    ns = sum(o[1] for o in slow) * 0.9
    print(f"fast reps {statistics.mean(o[0] for o in fast):.1f} us/step, slow {statistics.mean(o[0] for o in slow):.1f}")
    print(f"{'kernel':42s} {'fast avg':>9s} {'slow avg':>9s} {'fast us/step':>12s} {'slow us/step':>12s}")
    keys = sorted(set(kf) | set(ks), key=lambda k: -(sum(ks.get(k, [])) / ns - sum(kf.get(k, [])) / nf))
    for k in keys:
        a, b = kf.get(k, [0]), ks.get(k, [0])
        print(f"{k[:42]:42s} {statistics.mean(a):9.1f} {statistics.mean(b):9.1f} {sum(a) / nf:12.1f} {sum(b) / ns:12.1f}")

    def qstats(group):
        busy, gaps, span = collections.Counter(), collections.defaultdict(list), 0
        for _, _, rep in group:
            rep = rep[len(rep) // 10:]
            span += rep[-1][1] - rep[0][0]
            byq = collections.defaultdict(list)
            for s, e, k, q in rep:
                byq[q].append((s, e, k))
            for q, ks_ in byq.items():
                busy[q] += sum(e - s for s, e, _ in ks_)
                for (s0, e0, k0), (s1, e1, k1) in zip(ks_, ks_[1:]):
                    gaps[(q, k0, k1)].append((s1 - e0) / 1e3)
        return busy, gaps, span

    for label, group in (("fast", fast), ("slow", slow)):
        busy, gaps, span = qstats(group)
        print(f"{label}: " + ", ".join(f"queue {q} busy {busy[q] / span:.2f}" for q in sorted(busy)))
        top = sorted(gaps.items(), key=lambda kv: -sum(kv[1]))[:8]
        n = nf if label == "fast" else ns
        for (q, k0, k1), v in top:
            print(f"   queue {q}: {sum(v) / n:7.1f} us/step idle  after {k0[:30]} before {k1[:30]}")


if __name__ == "__main__":
    if sys.argv[1] == "--analyze":
        analyze(sys.argv[2])
    else:
        run()
