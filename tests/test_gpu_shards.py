"""Multi-GPU product path on one MI355X:
shard sessions (GhostmSessionCreateShard) each search one balanced, group-aligned
range of ONE query set; their outputs concatenated in rank order must be the
reference output, and their device hit records the unsharded records.

The 2-process test runs two real ranks (torch.distributed over gloo, both on
cuda:0, as the driver's 8-GPU run does over RCCL): each rank searches its shard,
the records go to rank 0 in the one gather, the text is assembled by rank 0, and
both are checked there."""
import hashlib
import json
import os
import socket
import subprocess
import sys
import textwrap

import numpy as np
import pytest

import cases
from ghostm_amd.aligner import HIT_DTYPE, Session
from ghostm_amd.shard import balanced_cuts

pytestmark = pytest.mark.gpu


def _argv(d, opts):
    return ["-i", f"{d}/q", "-d", f"{d}/db", "-o", f"{d}/x", "-D", "0"] + list(opts)


def _sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("ds,var,opts", [("syn_dna", "default", []), ("syn_small", "default", []),
                                         ("syn_chunks", "default", []), ("cfg2_20k", "default", []),
                                         ("syn_scale", "default", [])])
def test_shards_concatenate_to_reference(world, ds, var, opts, dataset, golden):
    d = dataset(ds)
    with Session(_argv(d, opts)) as s:
        s.run()
        full_hits = s.hits()
    texts, hits, ranges = [], [], []
    for r in range(world):
        with Session(_argv(d, opts), shard=(r, world)) as s:
            s.run()
            texts.append(s.output())
            hits.append(s.hits())
            dev = s.device_hits().cpu().numpy()
            assert dev.tobytes() == hits[-1].tobytes()
            ranges.append(s.shard_range())
    assert _sha(b"".join(texts)) == golden["aln"][f"{ds}/{var}"]["sha256"]
    assert np.concatenate(hits).tobytes() == full_hits.tobytes()
    assert ranges[0][0] == 0 and all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))


def test_more_shards_than_queries(dataset, golden):
    """protein_testset has 7 queries; with 10 shards some are empty and still run."""
    d = dataset("protein_testset")
    texts = []
    for r in range(10):
        with Session(_argv(d, []), shard=(r, 10)) as s:
            s.run()
            texts.append(s.output())
    assert _sha(b"".join(texts)) == golden["aln"]["protein_testset/y0"]["sha256"]
    assert sum(1 for t in texts if not t) >= 3


# batch-cut variants (-l in candidates via the test hook): the unsharded run cuts
# the chunk into several batches; every shard must replay those cuts (carried
# lists re-sorted per batch, batches splitting name groups, the dropped carried
# last query, the stop at an empty first batch: reference aligner.cpp:131-171,
# 511-514, 687-769). The oracle honours the same hook.
SHARD_BATCH = [
    ("syn_dna", "cut13", ["-y", "2"], {"GHOSTM_MAX_LIST_OVERRIDE": "13"}),
    ("syn_dna", "cut57_b3", ["-b", "3"], {"GHOSTM_MAX_LIST_OVERRIDE": "57"}),
    ("syn_dna", "cut100", [], {"GHOSTM_MAX_LIST_OVERRIDE": "100"}),
    ("syn_small", "cut300_b20", ["-b", "20", "-y", "2"], {"GHOSTM_MAX_LIST_OVERRIDE": "300"}),
    ("syn_small", "cut50", [], {"GHOSTM_MAX_LIST_OVERRIDE": "50"}),
    ("syn_small", "cut1", [], {"GHOSTM_MAX_LIST_OVERRIDE": "1"}),
    ("syn_repeat", "cut600_b20", ["-b", "20"], {"GHOSTM_MAX_LIST_OVERRIDE": "600"}),
    ("syn_chunks", "cut4000_b20", ["-b", "20", "-y", "2"], {"GHOSTM_MAX_LIST_OVERRIDE": "4000"}),
]


class _Env:
    def __init__(self, env):
        self.env = env

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.env}
        os.environ.update(self.env)

    def __exit__(self, *exc):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


_ORACLE_OUT = {}


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("ds,var,opts,env", SHARD_BATCH, ids=[f"{v[0]}/{v[1]}" for v in SHARD_BATCH])
def test_shards_replay_unsharded_batches(world, ds, var, opts, env, dataset, tmp_path):
    """Shards of a query set whose chunks need several batches: their rank-order
    concatenation equals the oracle's unsharded output, and their records the
    unsharded GPU records."""
    d = dataset(ds)
    key = (ds, var)
    if key not in _ORACLE_OUT:  # one oracle run per variant (syn_chunks takes a minute)
        _ORACLE_OUT[key] = cases.run_aln(cases.ORACLE, d, opts, env, str(tmp_path / "o.out"))
    want = _ORACLE_OUT[key]
    with _Env(env):
        with Session(_argv(d, opts)) as s:
            s.run()
            assert s.output() == want
            full_hits = s.hits()
            if var != "cut1":
                assert s.stats()["batches"] > 1
        texts, hits = [], []
        for r in range(world):
            with Session(_argv(d, opts), shard=(r, world)) as s:
                s.run()
                texts.append(s.output())
                hits.append(s.hits())
    assert b"".join(texts) == want
    assert np.concatenate(hits).tobytes() == full_hits.tobytes()


def _query_table(d):
    """Per query of chunk 0: residues (the shard weight) and names."""
    inf = np.fromfile(f"{d}/q_0.inf", dtype="<u4")
    nq, L = int(inf[0]), int(inf[1])
    seq = np.fromfile(f"{d}/q_0.seq", dtype=np.uint8)[: nq * L].reshape(nq, L)
    notx = seq != 23
    last = np.where(notx.any(axis=1), L - 1 - np.argmax(notx[:, ::-1], axis=1), 0)
    names = open(f"{d}/q_0.nam").read().split("\n")[:nq]
    return (last + 1).tolist(), names


def test_shard_starting_at_an_overflow_query(dataset, tmp_path):
    """A shard whose first query alone exceeds -l in the middle of the unsharded
    run: batching the shard on its own would end its chunk at once (the
    reference stops at an empty first batch); replaying the unsharded cuts keeps
    it. The world is picked so that such a cut exists."""
    d = dataset("syn_small")
    prefix = str(tmp_path / "dump")
    cases.run_aln(cases.ORACLE, d, [], {"GHOSTM_ORACLE_DUMP": prefix}, str(tmp_path / "all.out"))
    cand = np.fromfile(prefix + ".cand", dtype="<u4").reshape(-1, 4)
    weights, names = _query_table(d)
    counts = np.bincount(cand[:, 0], minlength=len(names))
    # a -l (in candidates) that the chunk's first query fits, and a world with a
    # cut at a query above it
    limit, world = next((lim, w) for lim in range(int(counts[0]), int(counts.max()))
                        for w in range(2, 65)
                        if any(counts[c] > lim for c in balanced_cuts(weights, names, w)[1:-1] if c < len(names)))
    env = {"GHOSTM_MAX_LIST_OVERRIDE": str(limit)}
    want = cases.run_aln(cases.ORACLE, d, [], env, str(tmp_path / "o.out"))
    assert want  # the unsharded run does not stop at its first query
    texts = []
    with _Env(env):
        for r in range(world):
            with Session(_argv(d, []), shard=(r, world)) as s:
                s.run()
                texts.append(s.output())
    assert b"".join(texts) == want


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


RANK = textwrap.dedent("""
    import json, os, sys
    import numpy as np
    import torch
    import torch.distributed as dist
    sys.path.insert(0, {repo!r})
    from ghostm_amd.aligner import HIT_DTYPE, Session
    from ghostm_amd.shard import gather_device_records, gather_bytes, torch_allgather
    rank, world, d, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    opts, local = json.loads(sys.argv[5]), sys.argv[6] == "local"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # local: the rank reads and counts only its own queries; the ranks agree on
    # the unsharded batch plan through the all-gather
    ex = torch_allgather(dist) if local else None
    with Session(["-i", d + "/q", "-d", d + "/db", "-o", d + "/x", "-D", "0"] + opts, shard=(rank, world),
                 exchange=ex) as s:
        s.run()
        recs = s.device_hits()            # on cuda:0
        text = s.output()
        lo, hi = s.shard_range()
    # the one data-path collective: hit records to rank 0 (gloo here: CPU tensors)
    parts = gather_device_records(recs.cpu(), dist, HIT_DTYPE.itemsize)
    texts = gather_bytes(text, dist)
    ranges = [None] * world
    dist.all_gather_object(ranges, (lo, hi))
    if rank == 0:
        with open(out + ".txt", "wb") as f:
            f.write(b"".join(texts))
        np.concatenate([p.numpy() for p in parts]).tofile(out + ".rec")
        json.dump(ranges, open(out + ".ranges", "w"))
    dist.barrier()
    dist.destroy_process_group()
""")


def _run_ranks(tmp_path, d, world, opts, env, local):
    script = tmp_path / "rank.py"
    script.write_text(RANK.format(repo=cases.REPO))
    out = str(tmp_path / "gathered")
    e = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), **env)
    procs = [subprocess.Popen([sys.executable, str(script), str(r), str(world), d, out, json.dumps(opts),
                               "local" if local else "self"], env=e,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(world)]
    logs = [p.communicate(timeout=300)[0].decode() for p in procs]
    assert all(p.returncode == 0 for p in procs), "\n".join(logs)
    recs = np.fromfile(out + ".rec", dtype=np.uint8).view(HIT_DTYPE)
    return open(out + ".txt", "rb").read(), recs, json.load(open(out + ".ranges"))


@pytest.mark.parametrize("local", [False, True], ids=["self", "local"])
@pytest.mark.parametrize("ds,var", [("syn_dna", "default"), ("syn_small", "default")])
def test_two_ranks_gather_to_rank0(ds, var, local, dataset, golden, tmp_path):
    d = dataset(ds)
    text, got, _ = _run_ranks(tmp_path, d, 2, [], {}, local)
    assert _sha(text) == golden["aln"][f"{ds}/{var}"]["sha256"]
    with Session(_argv(d, [])) as s:
        s.run()
        want = s.hits()
    assert got.tobytes() == want.tobytes()


@pytest.mark.parametrize("ds,var,opts,env,world", [
    ("syn_dna", "cut13", ["-y", "2"], {"GHOSTM_MAX_LIST_OVERRIDE": "13"}, 3),
    ("syn_small", "cut300_b20", ["-b", "20", "-y", "2"], {"GHOSTM_MAX_LIST_OVERRIDE": "300"}, 2),
    ("syn_small", "cut50", [], {"GHOSTM_MAX_LIST_OVERRIDE": "50"}, 8),
    ("syn_chunks", "cut4000_b20", ["-b", "20", "-y", "2"], {"GHOSTM_MAX_LIST_OVERRIDE": "4000"}, 3),
    ("syn_chunks", "default", [], {}, 8),
    ("protein_testset", "y0", [], {}, 10),  # more ranks than queries: empty ranks still exchange
    ("syn_chunks", "S1", ["-S", "1"], {}, 3),  # -S: the selected chunks only, global indices from there
], ids=lambda v: v if isinstance(v, str) else None)
def test_rank_local_shards_agree_on_the_batch_plan(ds, var, opts, env, world, dataset, golden, tmp_path):
    """Rank-local shard sessions (GhostmSessionCreateShardEx over gloo, every rank
    on cuda:0): each rank reads and counts only its queries, the all-gathered
    counts give the unsharded batch cuts, and the gathered text and records are
    the unsharded ones."""
    d = dataset(ds)
    if f"{ds}/{var}" in golden["aln"]:
        want_sha = golden["aln"][f"{ds}/{var}"]["sha256"]
    else:
        key = (ds, var)
        if key not in _ORACLE_OUT:
            _ORACLE_OUT[key] = cases.run_aln(cases.ORACLE, d, opts, env, str(tmp_path / "o.out"))
        want_sha = _sha(_ORACLE_OUT[key])
    text, got, ranges = _run_ranks(tmp_path, d, world, opts, env, True)
    assert _sha(text) == want_sha
    with _Env(env):
        with Session(_argv(d, opts)) as s:
            s.run()
            want = s.hits()
    assert got.tobytes() == want.tobytes()
    assert ranges[0][0] == 0 and all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))


def test_rank_local_names_file_shorter_than_the_chunk(dataset, tmp_path):
    """A .nam with fewer lines than the chunk's queries: the reference reads the
    missing names as empty (query_reader.cpp, ReadNameLines' getline path), and a
    rank-local shard reads its names the same way (QueryChunkIndex falls back to
    the full name list), so shards still concatenate to the unsharded output."""
    import shutil

    src = dataset("syn_small")
    d = tmp_path / "ds"
    shutil.copytree(src, d)
    lines = (d / "q_0.nam").read_bytes().split(b"\n")
    (d / "q_0.nam").write_bytes(b"\n".join(lines[:-6]))  # last names missing, last line unterminated
    with Session(_argv(str(d), [])) as s:
        s.run()
        want = s.output()
        want_hits = s.hits()
    assert want
    text, got, _ = _run_ranks(tmp_path, str(d), 3, [], {}, True)
    assert text == want
    assert got.tobytes() == want_hits.tobytes()


FAIL_RANK = textwrap.dedent("""
    import datetime, sys
    import torch.distributed as dist
    sys.path.insert(0, {repo!r})
    from ghostm_amd.aligner import Session
    from ghostm_amd.shard import torch_allgather
    rank, world, d, other = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    mode = sys.argv[5]
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=240))
    q, db = d + "/q", d + "/db"
    if rank == 1 and mode == "missing_db":
        db = d + "/no_such_db"
    if rank == 1 and mode == "other_queries":
        q = other + "/q"
    try:
        Session(["-i", q, "-d", db, "-o", d + "/x", "-D", "0"], shard=(rank, world), exchange=torch_allgather(dist))
    except Exception as e:
        print("create failed:", e, flush=True)
        sys.exit(3)
    print("create succeeded", flush=True)
""")


@pytest.mark.parametrize("mode,msg", [("missing_db", "failed at creation"),
                                      ("other_queries", "sees a different query/DB set")])
def test_rank_local_creation_fails_on_every_rank(mode, msg, dataset, tmp_path):
    """One rank that cannot load (a missing DB) or that sees another query set
    makes every rank's GhostmSessionCreateShardEx fail through the creation
    header exchange, instead of its peers waiting in the plan's all-gather."""
    d, other = dataset("syn_small"), dataset("syn_dna")
    script = tmp_path / "fail_rank.py"
    script.write_text(FAIL_RANK.format(repo=cases.REPO))
    e = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    procs = [subprocess.Popen([sys.executable, str(script), str(r), "3", d, other, mode], env=e,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(3)]
    logs = [p.communicate(timeout=200)[0].decode() for p in procs]
    assert all(p.returncode == 3 for p in procs), "\n".join(logs)
    for r, log in enumerate(logs):
        if r != 1:
            assert msg in log, log


@pytest.mark.parametrize("name,world", [("cfg4_20k_l1_b20y2", 3), ("dna40k_l1_b20", 8)])
def test_rank_local_multi_batch_matches_reference_pin(name, world, tmp_path):
    """Rank-local shard sessions over gloo (GhostmSessionCreateShardEx, every
    rank on cuda:0) on a workload the reference cut into several batches
    (`-l 1`, one reference process): the gathered text is the reference's."""
    from ghostm_amd import workloads

    with open(os.path.join(cases.GOLDEN, "full_golden.json")) as f:
        pin = json.load(f).get(name)
    if pin is None:
        pytest.skip(f"{name} not pinned")
    d = str(tmp_path / "ds")
    workloads.make_db(name, d)
    workloads.make_queries(name, d)
    text, got, ranges = _run_ranks(tmp_path, d, world, workloads.WORKLOADS[name]["aln"], {}, True)
    assert len(text) == pin["bytes"]
    assert _sha(text) == pin["sha256"]
    assert ranges[0][0] == 0 and all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
