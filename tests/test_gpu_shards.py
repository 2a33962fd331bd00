"""Multi-GPU product path on one MI355X:
shard sessions (GhostmSessionCreateShard) each search one balanced, group-aligned
range of ONE query set; their outputs concatenated in rank order must be the
reference output, and their device hit records the unsharded records.

The 2-process test runs two real ranks (torch.distributed over gloo, both on
cuda:0, as the driver's 8-GPU run does over RCCL): each rank searches its shard,
the records go to rank 0 in the one gather, the text is assembled by rank 0, and
both are checked there."""
import hashlib
import os
import socket
import subprocess
import sys
import textwrap

import numpy as np
import pytest

import cases
from ghostm_amd.aligner import HIT_DTYPE, Session

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


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


RANK = textwrap.dedent("""
    import hashlib, os, sys
    import numpy as np
    import torch
    import torch.distributed as dist
    sys.path.insert(0, {repo!r})
    from ghostm_amd.aligner import HIT_DTYPE, Session
    from ghostm_amd.shard import gather_device_records, gather_bytes
    rank, world, d, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    dist.init_process_group("gloo", rank=rank, world_size=world)
    with Session(["-i", d + "/q", "-d", d + "/db", "-o", d + "/x", "-D", "0"], shard=(rank, world)) as s:
        s.run()
        recs = s.device_hits()            # on cuda:0
        text = s.output()
    # the one data-path collective: hit records to rank 0 (gloo here: CPU tensors)
    parts = gather_device_records(recs.cpu(), dist, HIT_DTYPE.itemsize)
    texts = gather_bytes(text, dist)
    if rank == 0:
        with open(out + ".txt", "wb") as f:
            f.write(b"".join(texts))
        np.concatenate([p.numpy() for p in parts]).tofile(out + ".rec")
    dist.barrier()
    dist.destroy_process_group()
""")


@pytest.mark.parametrize("ds,var", [("syn_dna", "default"), ("syn_small", "default")])
def test_two_ranks_gather_to_rank0(ds, var, dataset, golden, tmp_path):
    d = dataset(ds)
    script = tmp_path / "rank.py"
    script.write_text(RANK.format(repo=cases.REPO))
    out = str(tmp_path / "gathered")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    procs = [subprocess.Popen([sys.executable, str(script), str(r), "2", d, out], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(2)]
    logs = [p.communicate(timeout=300)[0].decode() for p in procs]
    assert all(p.returncode == 0 for p in procs), "\n".join(logs)
    text = open(out + ".txt", "rb").read()
    assert _sha(text) == golden["aln"][f"{ds}/{var}"]["sha256"]
    with Session(_argv(d, [])) as s:
        s.run()
        want = s.hits()
    got = np.fromfile(out + ".rec", dtype=np.uint8).view(HIT_DTYPE)
    assert got.tobytes() == want.tobytes()
