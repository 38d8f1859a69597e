"""bench.py --gpus N starts its own N ranks when no launcher did (langsplat_amd/launch.py; VERDICT r05
missing item 1): the per-rank environment, the decision, the exit status, and real child ranks that
rendezvous over gloo from that environment alone.  CPU only."""
import os
import sys
import time

import pytest
import torch

from langsplat_amd import launch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_should_launch_only_outside_a_launcher():
    assert not launch.should_launch(1, {})
    assert launch.should_launch(2, {})
    assert launch.should_launch(8, {"LOCAL_RANK": "0"})  # a stray LOCAL_RANK alone is no process group
    assert not launch.should_launch(8, {"WORLD_SIZE": "8", "RANK": "3"})  # torchrun's ranks
    assert not launch.should_launch(2, {"RANK": "0"})


def test_rank_envs_match_torchrun():
    base = {"PATH": "/bin", "RANK": "5", "WORLD_SIZE": "9", "MASTER_PORT": "1", "LSR_DIST_BACKEND": "gloo"}
    envs = launch.rank_envs(4, 29611, base)
    assert len(envs) == 4
    for r, e in enumerate(envs):
        assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"], e["LOCAL_WORLD_SIZE"]) == (str(r), str(r), "4", "4")
        assert (e["MASTER_ADDR"], e["MASTER_PORT"], e["GROUP_RANK"]) == ("127.0.0.1", "29611", "0")
        assert e["PATH"] == "/bin" and e["LSR_DIST_BACKEND"] == "gloo"  # the rest passes through
    assert base["RANK"] == "5"  # the caller's mapping is not modified
    with pytest.raises(ValueError):
        launch.rank_envs(0, 29611, base)
    with pytest.raises(ValueError):
        launch.rank_envs(2, 0, base)


def test_worst_status():
    assert launch.worst_status([0, 0, 0]) == 0
    assert launch.worst_status([0, 3, 1]) == 3
    assert launch.worst_status([0, -9]) == 137  # killed by SIGKILL, as a shell reports it


_CHILD = """
import os, sys, torch, torch.distributed as dist
dist.init_process_group("gloo")
t = torch.tensor([float(dist.get_rank() + 1)])
dist.all_reduce(t)
with open(os.path.join(sys.argv[1], "rank%s" % os.environ["RANK"]), "w") as f:
    f.write("%d %d %s %g" % (dist.get_rank(), dist.get_world_size(), os.environ["LOCAL_RANK"], t.item()))
dist.destroy_process_group()
"""


@pytest.mark.parametrize("n", [2, 4])
def test_launch_runs_n_ranks_that_rendezvous(tmp_path, n):
    rc = launch.launch(["-c", _CHILD, str(tmp_path)], n)
    assert rc == 0
    for r in range(n):
        rank, world, local, total = open(tmp_path / f"rank{r}").read().split()
        assert (int(rank), int(world), int(local)) == (r, n, r)
        assert float(total) == n * (n + 1) / 2


def test_launch_stops_the_others_when_one_rank_fails():
    code = "import os, sys, time\nif os.environ['RANK'] == '1': sys.exit(3)\ntime.sleep(120)"
    t0 = time.monotonic()
    assert launch.launch(["-c", code], 3, grace_s=5.0) == 3
    assert time.monotonic() - t0 < 30  # the sleeping ranks were stopped, not waited for


def test_bench_launches_before_touching_the_gpu(monkeypatch):
    """A plain `python bench.py --gpus 2` hands over to the launcher at the top of main(), with its own
    path and arguments, and exits with the launcher's status."""
    import bench
    seen = {}

    def fake(argv, n):
        seen["argv"], seen["n"] = list(argv), n
        seen["cuda_initialized"] = torch.cuda.is_initialized()
        return 7

    for k in ("WORLD_SIZE", "RANK"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setattr(bench.launch, "launch", fake)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "10"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7
    assert seen["n"] == 2 and seen["argv"][0] == os.path.join(ROOT, "bench.py")
    assert seen["argv"][1:] == ["--gpus", "2", "--steps", "10"]
    assert not seen["cuda_initialized"]


def test_bench_refuses_a_world_that_is_not_gpus(monkeypatch):
    import bench
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    with pytest.raises(SystemExit, match="--gpus 2 but the process group has 1"):
        bench.main()
