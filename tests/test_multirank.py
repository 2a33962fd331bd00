"""Multi-GPU path on CPU: shard cuts at name-group boundaries,
the single gather of hit records over a real torch.distributed process group
(gloo, world size 2 — the GPU run uses the same code over RCCL), and that
sharded searches concatenated in rank order give the unsharded output."""
import os
import socket
import subprocess
import sys
import textwrap

import numpy as np

import cases
from ghostm_amd.aligner import HIT_DTYPE
from ghostm_amd.shard import balanced_cuts


def test_balanced_cuts_never_split_a_name_group():
    names = ["a"] * 6 + ["b"] * 6 + ["c"] + ["d"] * 6 + ["e"] * 2
    weights = [10] * len(names)
    for world in (1, 2, 3, 4, 8):
        cuts = balanced_cuts(weights, names, world)
        assert cuts[0] == 0 and cuts[-1] == len(names) and len(cuts) == world + 1
        assert all(x <= y for x, y in zip(cuts, cuts[1:]))
        for c in cuts[1:-1]:
            assert c == len(names) or c == 0 or names[c] != names[c - 1]
    cuts = balanced_cuts([1] * 100, [str(i) for i in range(100)], 4)
    assert cuts == [0, 25, 50, 75, 100]


def test_native_shard_cuts_equal_python_rule(built):
    """GhostmShardCuts (used by the shard sessions, C ABI, host only) cuts exactly
    where balanced_cuts does, on random weights and name-group structures."""
    from ghostm_amd.shard import shard_cuts_native

    rng = np.random.default_rng(5)
    for trial in range(300):
        n = int(rng.integers(0, 60))
        weights = rng.integers(1, 128, size=n)
        names, g = [], 0
        for i in range(n):
            if i == 0 or rng.random() < 0.6:
                g += 1
            names.append(str(g))
        starts = [1 if i == 0 or names[i] != names[i - 1] else 0 for i in range(n)]
        for world in (1, 2, 3, 7, 8, 70):
            assert shard_cuts_native(weights, starts, world) == balanced_cuts(list(weights), names, world), \
                (trial, world)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


WORKER = textwrap.dedent("""
    import os, sys
    import numpy as np
    import torch.distributed as dist
    sys.path.insert(0, {repo!r})
    from ghostm_amd.aligner import HIT_DTYPE
    import torch
    from ghostm_amd.shard import gather_device_records, gather_hits
    rank, world = int(sys.argv[1]), int(sys.argv[2])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = [3, 0, 5][rank]  # rank 1 holds no hits
    h = np.zeros(n, dtype=HIT_DTYPE)
    h["query_id"] = rank * 100 + np.arange(n)
    h["seq_id"] = 0.25 * rank
    out = gather_hits(h, dist, "cpu")
    # the device-record form (uint8 payload tensors; CPU tensors over gloo here)
    dev = gather_device_records(torch.from_numpy(h.view(np.uint8).copy()), dist, HIT_DTYPE.itemsize)
    if rank == 0:
        np.save(sys.argv[3], np.concatenate(out))
        assert [len(x) for x in out] == [3, 0, 5][:world]
        flat = np.concatenate([t.numpy() for t in dev]).view(HIT_DTYPE)
        assert flat.tobytes() == np.concatenate(out).tobytes()
    dist.barrier()
    dist.destroy_process_group()
""")


def test_gather_hits_over_gloo(tmp_path):
    for world in (2, 3):
        script = tmp_path / "worker.py"
        script.write_text(WORKER.format(repo=cases.REPO))
        out = tmp_path / f"gathered{world}.npy"
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
        procs = [subprocess.Popen([sys.executable, str(script), str(r), str(world), str(out)], env=env,
                                  stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(world)]
        logs = [p.communicate(timeout=180)[0].decode() for p in procs]
        assert all(p.returncode == 0 for p in procs), "\n".join(logs)
        got = np.load(out)
        assert got.dtype == HIT_DTYPE
        want_q = [0, 1, 2] + ([200, 201, 202, 203, 204] if world == 3 else [])
        assert got["query_id"].tolist() == want_q
        assert got["seq_id"].tolist() == [0.0] * 3 + ([0.5] * 5 if world == 3 else [])


AG_WORKER = textwrap.dedent("""
    import sys
    import torch.distributed as dist
    sys.path.insert(0, {repo!r})
    from ghostm_amd.shard import torch_allgather
    rank, world = int(sys.argv[1]), int(sys.argv[2])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ag = torch_allgather(dist)
    sizes = [(3 * r) % 5 for r in range(world)]  # rank 0 and others send nothing
    mine = bytes((rank * 16 + k) % 256 for k in range(sizes[rank]))
    got = ag(mine, sizes)
    want = b"".join(bytes((r * 16 + k) % 256 for k in range(sizes[r])) for r in range(world))
    assert got == want, (got, want)
    assert ag(b"", [0] * world) == b""
    dist.barrier()
    dist.destroy_process_group()
""")


def test_torch_allgather_over_gloo(tmp_path):
    """The all-gather rank-local shard sessions agree on their batch plan with
    (GhostmAllGatherFn through Session(exchange=...)): ragged per-rank sizes,
    empty ranks, rank order."""
    for world in (2, 3):
        script = tmp_path / "ag.py"
        script.write_text(AG_WORKER.format(repo=cases.REPO))
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
        procs = [subprocess.Popen([sys.executable, str(script), str(r), str(world)], env=env,
                                  stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(world)]
        logs = [p.communicate(timeout=180)[0].decode() for p in procs]
        assert all(p.returncode == 0 for p in procs), "\n".join(logs)


def _read_fasta(path):
    recs, name, seq = [], None, []
    with open(path) as f:
        for line in f:
            if line.startswith(">"):
                if name is not None:
                    recs.append((name, "".join(seq)))
                name, seq = line[1:].rstrip("\n"), []
            else:
                seq.append(line.strip())
    if name is not None:
        recs.append((name, "".join(seq)))
    return recs


def test_sharded_search_concatenates_to_unsharded_output(dataset, tmp_path):
    """Each rank formats and searches its own contiguous read range; rank-order
    concatenation of the outputs is the single-process output (DNA reads: every
    read's six frames form one name group and stay on one shard). Checked with
    the CPU oracle so it runs without a GPU."""
    d = dataset("syn_dna")
    full = cases.run_aln(cases.ORACLE, d, [], {}, str(tmp_path / "full.out"))
    reads = _read_fasta(os.path.join(d, "q.fa"))
    cuts = balanced_cuts([len(s) for _, s in reads], [n for n, _ in reads], 3)
    parts = []
    for r in range(3):
        sd = tmp_path / f"shard{r}"
        sd.mkdir()
        with open(sd / "q.fa", "w") as f:
            for name, seq in reads[cuts[r]:cuts[r + 1]]:
                f.write(f">{name}\n{seq}\n")
        subprocess.run([cases.GHOSTM, "qry", "-i", str(sd / "q.fa"), "-o", str(sd / "q"), "-t", "d", "-l", "150"],
                       check=True, capture_output=True)
        out = sd / "o.out"
        subprocess.run([cases.ORACLE, "aln", "-i", str(sd / "q"), "-d", os.path.join(d, "db"), "-o", str(out)],
                       check=True, capture_output=True)
        parts.append(out.read_bytes())
    assert b"".join(parts) == full
    assert all(parts)
