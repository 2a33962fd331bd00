"""`bench.py --gpus N` launching its own ranks (ghostm_amd/launch.py), on CPU over
gloo: children get the torchrun environment, rank 0's line is the output, a
failing rank stops every rank (ok-flag agreement) instead of hanging them, a
WORLD_SIZE that disagrees with --gpus is refused, the per-rank CPU placement,
and the fixed-capacity record gather (the one data-path collective)."""
import json
import os
import subprocess
import sys
import textwrap
import time

import pytest

from ghostm_amd import launch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import datetime, json, os, sys
    sys.path.insert(0, {repo!r})
    import torch, torch.distributed as dist
    from ghostm_amd import launch
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    assert os.environ["LOCAL_RANK"] == str(rank) and os.environ["LOCAL_WORLD_SIZE"] == str(world)
    assert os.environ["MASTER_ADDR"] == "127.0.0.1"
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=60))
    mode = sys.argv[1]
    for step in range(3):
        ok = True
        try:
            if mode == "fail" and rank == 1 and step == 1:
                raise RuntimeError("rank 1 fails in step 1")
        except RuntimeError:
            launch.agree(dist, False, "cpu", "step")
            raise
        launch.agree(dist, True, "cpu", "step")
    t = torch.tensor([rank + 1])
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({{"world": world, "sum": int(t.item())}}), flush=True)
    dist.destroy_process_group()
""")


def _run_spawn(tmp_path, n, mode, timeout=120):
    child = tmp_path / "child.py"
    child.write_text(CHILD.format(repo=REPO))
    code = (f"import sys; sys.path.insert(0, {REPO!r}); from ghostm_amd import launch; "
            f"sys.exit(launch.spawn([{str(child)!r}, {mode!r}], {n}, grace_s=20))")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=timeout, env=env)
    return p, time.monotonic() - t0


def test_spawn_starts_ranks_and_forwards_rank0_line(tmp_path):
    p, _ = _run_spawn(tmp_path, 3, "ok")
    assert p.returncode == 0, p.stderr
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert lines == [{"world": 3, "sum": 6}]


def test_failing_rank_stops_every_rank(tmp_path):
    p, dt = _run_spawn(tmp_path, 3, "fail")
    assert p.returncode != 0
    assert "rank 1 fails in step 1" in p.stderr
    # the peers leave through the ok-flag agreement, not the 60 s gloo timeout
    assert "another rank failed in step" in p.stderr
    assert dt < 50, dt
    assert not [x for x in p.stdout.splitlines() if x.startswith("{")]


def test_world_from_env(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert launch.world_from_env(None) == (1, False)
    assert launch.world_from_env(1) == (1, False)
    assert launch.world_from_env(8) == (8, True)
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert launch.world_from_env(4) == (4, False)
    assert launch.world_from_env(None) == (4, False)
    with pytest.raises(SystemExit):
        launch.world_from_env(8)


def test_bench_refuses_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "3", "--steps", "1"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode != 0
    assert "--gpus 3 but WORLD_SIZE=2" in p.stderr


def test_cpu_lists_and_shares():
    assert launch.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert launch._fmt_cpulist([0, 1, 2, 3, 8, 10, 11]) == "0-3,8,10-11"
    cpus = list(range(10))
    parts = [launch.split_share(cpus, 3, i) for i in range(3)]
    assert parts == [[0, 1, 2, 3], [4, 5, 6], [7, 8, 9]]
    assert [launch.split_share([0, 1], 3, i) for i in range(3)] == [[0], [1], [0]]


PLACE = textwrap.dedent("""
    import datetime, json, os, sys
    sys.path.insert(0, {repo!r})
    import torch.distributed as dist
    from ghostm_amd import launch
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=60))
    info = launch.bind_numa(dist, dist.get_rank(), 0)
    info["affinity"] = sorted(os.sched_getaffinity(0))
    # every thread, including those gloo started before the binding
    info["thread_affinity"] = [sorted(os.sched_getaffinity(int(t))) for t in os.listdir("/proc/self/task")]
    info["env_threads"] = os.environ["GHOSTM_THREADS"]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, info)
    if dist.get_rank() == 0:
        print(json.dumps(out), flush=True)
    dist.destroy_process_group()
""")


def test_bind_numa_gives_disjoint_cpu_shares(tmp_path):
    """No GPU here: the placement falls back to the allowed CPUs, split
    disjointly among the ranks that share them."""
    child = tmp_path / "place.py"
    child.write_text(PLACE.format(repo=REPO))
    code = (f"import sys; sys.path.insert(0, {REPO!r}); from ghostm_amd import launch; "
            f"sys.exit(launch.spawn([{str(child)!r}], 2, grace_s=20))")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 0, p.stderr
    out = json.loads([x for x in p.stdout.splitlines() if x.startswith("[{")][0])
    a, b = out[0]["affinity"], out[1]["affinity"]
    allowed = sorted(os.sched_getaffinity(0))
    if len(allowed) >= 2:
        assert not set(a) & set(b)
        assert sorted(a + b) == allowed
    for o in out:
        assert o["ranks_sharing_cpus"] == 2
        assert int(o["env_threads"]) == o["threads"] >= 1
        assert o["bound"] and o["threads_bound"] > 1  # the backend's threads too
        assert all(t == o["affinity"] for t in o["thread_affinity"]), o["thread_affinity"]


GATHER = textwrap.dedent("""
    import datetime, os, sys
    sys.path.insert(0, {repo!r})
    import torch, torch.distributed as dist
    from ghostm_amd.shard import RecordGather
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=60))
    rank, world = dist.get_rank(), dist.get_world_size()
    g = RecordGather(dist, 7, 32, "cpu")
    for step, counts in enumerate(([3, 0, 7], [7, 5, 1])):
        n = counts[rank]
        recs = torch.arange(n * 32, dtype=torch.int32).to(torch.uint8) + (rank * 16 + step)
        g.payload()[: n * 32].copy_(recs)
        g.set_count(n)
        g.gather()
        if rank == 0:
            parts = g.records()
            assert [p.numel() // 32 for p in parts] == counts, parts
            for r, p in enumerate(parts):
                want = torch.arange(counts[r] * 32, dtype=torch.int32).to(torch.uint8) + (r * 16 + step)
                assert torch.equal(p, want)
    try:
        g.set_count(8)
        raise SystemExit("over capacity accepted")
    except ValueError:
        pass
    dist.destroy_process_group()
""")


def test_record_gather_over_gloo(tmp_path):
    child = tmp_path / "gather.py"
    child.write_text(GATHER.format(repo=REPO))
    code = (f"import sys; sys.path.insert(0, {REPO!r}); from ghostm_amd import launch; "
            f"sys.exit(launch.spawn([{str(child)!r}], 3, grace_s=20))")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 0, p.stderr
