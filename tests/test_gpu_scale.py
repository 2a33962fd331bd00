"""GPU parity at the scale the headline workload runs:

* every K1 size class (the LDS hash kernels of classes 0-2 and the global
  merge of class 3) and the >slot offset pass, shown to run by the session's
  per-class counters, against the reference golden;
* the device-merge pipeline cut into many segments with a shrinking tail (the
  path every cfg3/cfg4 run takes), on small datasets and on the cfg4 generator's
  own DB;
* the FULL BASELINE workloads (cfg2 substitute, cfg3, cfg4, cfg5), whose complete
  output is compared with the sha256 of the reference CPU program's output
  (tests/golden/full_golden.json, tests/golden/make_full_golden.py).
"""
import hashlib
import json
import os

import numpy as np
import pytest

import cases
from ghostm_amd import workloads
from ghostm_amd.aligner import Session

pytestmark = pytest.mark.gpu


def _run(d, opts, env, qprefix="q", dprefix="db"):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        with Session(["-i", os.path.join(d, qprefix), "-d", os.path.join(d, dprefix), "-o", os.path.join(d, "x"),
                      "-D", "0"] + list(opts)) as s:
            s.run()
            text, st, hits = s.output(), s.stats(), s.hits()
            dev = s.device_hits().cpu().numpy()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return text, st, hits, dev


def _sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def _caps(d):
    """Class caps at the quartiles of the dataset's K1 list-entry counts, so that
    each of the four classes receives about a quarter of the queries."""
    n = cases.k1_list_entries(d)
    q = [int(np.percentile(n[n > 0], p)) for p in (25, 50, 75)]
    return ",".join(str(x) for x in q)


@pytest.mark.parametrize("k1", ["hash", "merge", "lists_only"])
@pytest.mark.parametrize("ds,var,opts", [("syn_small", "default", []), ("syn_dna", "default", []),
                                         ("syn_short", "default", []), ("syn_chunks", "default", []),
                                         ("syn_small", "r4", ["-r", "4"])])
def test_every_k1_class_and_the_offset_pass(k1, ds, var, opts, dataset, golden):
    """GHOSTM_K1_CAPS lowers the class caps to the dataset's quartiles and
    GHOSTM_K1_SLOT_CAP shrinks the slot to 2 candidates: all four classes and the
    offset pass for wide queries run, in the hash (default) and merge K1 forms,
    and with every class launched from host lists (GHOSTM_K1_EARLY=0: no class
    launched over all queries before the host class pass)."""
    d = dataset(ds)
    env = {"GHOSTM_K1_CAPS": _caps(d), "GHOSTM_K1_SLOT_CAP": "2"}
    if k1 == "merge":
        env["GHOSTM_K1"] = "merge"
    if k1 == "lists_only":
        env["GHOSTM_K1_EARLY"] = "0"
    text, st, hits, dev = _run(d, opts, env)
    assert _sha(text) == golden["aln"][f"{ds}/{var}"]["sha256"]
    for c in range(4):
        assert st[f"seed_queries_class{c}"] > 0, (c, st)
    assert st["seed_queries_wide"] > 0
    assert (st["seed_runs_hash"] == 0) if k1 == "merge" else (st["seed_runs_hash"] > 0)
    assert dev.tobytes() == hits.tobytes()


@pytest.mark.parametrize("devoff", ["1", "0"])
@pytest.mark.parametrize("ds,var,opts", [("syn_small", "default", []), ("syn_dna", "default", []),
                                         ("syn_scale", "default", []), ("syn_chunks", "default", [])])
def test_k1_overflow_redo_and_device_offsets(devoff, ds, var, opts, dataset, golden):
    """K1's filter-queue overflow path, forced on every third query of the LDS
    classes (GHOSTM_K1_FORCE_OVERFLOW): the unfiltered table redoes them, the host
    offsets replace the device ones and the compaction runs again; with the
    device offsets on (default) and off (GHOSTM_K1_DEVOFF=0). Same bytes as the
    reference."""
    d = dataset(ds)
    text, st, hits, dev = _run(d, opts, {"GHOSTM_K1_FORCE_OVERFLOW": "3", "GHOSTM_K1_DEVOFF": devoff})
    assert _sha(text) == golden["aln"][f"{ds}/{var}"]["sha256"]
    assert st["seed_filter_overflows"] > 0, st
    assert dev.tobytes() == hits.tobytes()


@pytest.mark.parametrize("windows", ["0", "1"])
@pytest.mark.parametrize("k1", ["filter", "hash"])
@pytest.mark.parametrize("ds,var,opts", [("syn_small", "default", []), ("syn_dna", "default", []),
                                         ("syn_scale", "default", []),
                                         ("syn_small", "b20_t1", ["-b", "20", "-t", "1", "-y", "2"])])
def test_k1_table_probe_bound_redo(windows, k1, ds, var, opts, dataset, golden):
    """K1's LDS bin table gives up after a bounded probe (BinTable: every bucket
    once at most) instead of looping; a query whose insert finds no room is
    marked kOverflow and redone by a table-free kernel. GHOSTM_K1_PROBE_WINDOWS
    lowers the bound: 0 fails every insert (every LDS-class query goes filter ->
    k_seed_hash -> k_seed merge, or k_seed_hash -> k_seed without the filter:
    GHOSTM_K1=hash, and -t 1: no filter below threshold 2), 1 fails only the bins whose first window is full.
    Same bytes as the reference either way (the round-5 hang: a bucket outside
    the table made the old unbounded probe spin forever)."""
    d = dataset(ds)
    env = {"GHOSTM_K1_PROBE_WINDOWS": windows}
    if k1 == "hash":
        env["GHOSTM_K1"] = "hash"
    text, st, hits, dev = _run(d, opts, env)
    assert _sha(text) == golden["aln"][f"{ds}/{var}"]["sha256"]
    assert dev.tobytes() == hits.tobytes()
    if windows == "0":
        assert st["seed_table_full"] > 0, st
        if k1 == "filter" and var != "b20_t1":  # the filter runs for thresholds >= 2
            assert st["seed_filter_overflows"] > 0, st


@pytest.mark.parametrize("ds,var,opts", [("syn_small", "default", []), ("syn_scale", "default", []),
                                         ("syn_chunks", "default", [])])
def test_k1_compaction_with_short_candidate_buffers(ds, var, opts, dataset, golden):
    """The device compaction behind K1's count read-back runs before the host
    knows the total: with room for fewer candidates than the run has
    (GHOSTM_K1_CAND_CAP), it writes only the queries that fit, and the host
    re-runs the copy into the grown buffers. Same bytes as the reference."""
    d = dataset(ds)
    text, st, hits, dev = _run(d, opts, {"GHOSTM_K1_CAND_CAP": "64"})
    assert _sha(text) == golden["aln"][f"{ds}/{var}"]["sha256"]
    assert st["seed_compact_redo"] > 0, st
    assert dev.tobytes() == hits.tobytes()


def test_device_pool_out_of_memory_retry(dataset, golden):
    """Blocks of destroyed sessions stay cached (DevPool); an allocation that
    runs out of memory empties the cache and retries (GHOSTM_DEV_OOM_TEST fails
    the first attempt whenever blocks are cached), and GhostmDevicePoolTrim
    frees the cache on request."""
    from ghostm_amd import native

    small, scale = dataset("syn_small"), dataset("syn_scale")
    native.load().GhostmDevicePoolTrim()
    text, _, _, _ = _run(small, [], {})
    assert _sha(text) == golden["aln"]["syn_small/default"]["sha256"]
    cached, retries0 = native.device_pool_info()
    assert cached > 0
    text, _, _, _ = _run(scale, [], {"GHOSTM_DEV_OOM_TEST": "1"})
    assert _sha(text) == golden["aln"]["syn_scale/default"]["sha256"]
    _, retries1 = native.device_pool_info()
    assert retries1 > retries0
    assert native.load().GhostmDevicePoolTrim() > 0
    assert native.device_pool_info()[0] == 0


def test_syn_scale_runs_the_cfg4_classes(dataset, golden):
    """The cfg4 generator's DB with its first 5000 queries, default options: K1
    classes 1 and 2 (k_seed_hash<512,12288>, <1024,24576>) and the offset pass
    run without any knob, and the output is the reference's."""
    d = dataset("syn_scale")
    text, st, hits, dev = _run(d, [], {})
    assert _sha(text) == golden["aln"]["syn_scale/default"]["sha256"]
    assert st["seed_queries_class1"] > 0 and st["seed_queries_class2"] > 0
    assert st["seed_queries_wide"] > 0
    assert st["seed_runs_hash"] > 0
    assert dev.tobytes() == hits.tobytes()


@pytest.mark.parametrize("ds,var,opts", [("syn_repeat", "default", []), ("syn_repeat", "b20_y2", ["-b", "20", "-y", "2"])])
def test_low_complexity_reaches_class3(ds, var, opts, dataset, golden):
    """Poly-Q / AKE-repeat queries have > 16384 K1 list entries (class 3, the
    global merge) and ~1000 candidates each, with tied scores: no knob needed."""
    d = dataset(ds)
    text, st, hits, dev = _run(d, opts, {})
    assert _sha(text) == golden["aln"][f"{ds}/{var}"]["sha256"]
    assert st["seed_queries_class3"] > 0 and st["seed_queries_wide"] > 0
    assert dev.tobytes() == hits.tobytes()


@pytest.mark.parametrize("ds,var,opts,seg,tail", [
    ("syn_small", "default", [], 300, 40),
    ("syn_small", "b20_t1", ["-b", "20", "-t", "1", "-y", "2"], 1000, 100),
    ("syn_dna", "default", [], 200, 30),
    ("syn_short", "default", [], 500, 50),
    ("syn_scale", "default", [], 100_000, 20_000),
    ("syn_repeat", "default", [], 400, 64),
    ("cfg2_20k", "default", [], 5000, 1000),
])
def test_many_segment_device_pipeline(ds, var, opts, seg, tail, dataset, golden):
    """The device-merge path cut into many segments (GHOSTM_SEGMENT_CANDS) with
    the 3/5 shrinking tail down to GHOSTM_TAIL_CANDS, the next segment's K2
    tasks prepared during the current K2, and per-segment device records: same
    text as the reference, same device records as host records."""
    d = dataset(ds)
    text, st, hits, dev = _run(d, opts, {"GHOSTM_SEGMENT_CANDS": str(seg), "GHOSTM_TAIL_CANDS": str(tail)})
    assert _sha(text) == golden["aln"][f"{ds}/{var}"]["sha256"]
    assert st["segments"] >= 4, st["segments"]
    assert dev.tobytes() == hits.tobytes()


@pytest.mark.parametrize("merge", ["device", "host"])
@pytest.mark.parametrize("ds,var,opts", [("syn_small", "default", []), ("syn_dna", "default", []),
                                         ("syn_chunks", "default", [])])
def test_streamed_output_file(merge, ds, var, opts, dataset, golden, tmp_path):
    """GhostmSessionRunToFile writes the -o file while the search runs (each
    segment's text as soon as it is formatted, in order): the file is the
    reference output over many segments, on the device-merge and host-merge
    paths, and a later write() leaves it as it is."""
    d = dataset(ds)
    env = {"GHOSTM_SEGMENT_CANDS": "300", "GHOSTM_TAIL_CANDS": "40"}
    if merge == "host":
        env["GHOSTM_MERGE"] = "host"
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    out = tmp_path / "streamed.out"
    out.write_bytes(b"stale bytes that must be truncated " * 1000)
    try:
        with Session(["-i", os.path.join(d, "q"), "-d", os.path.join(d, "db"), "-o", str(out), "-D", "0"]
                     + list(opts)) as s:
            s.run(to_file=True)
            text = s.output()
            assert out.read_bytes() == text
            s.write()
            assert out.read_bytes() == text
            s.run()  # a plain run after a streamed one: write() writes again
            out.unlink()
            s.write()
            assert out.read_bytes() == text
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert _sha(text) == golden["aln"][f"{ds}/{var}"]["sha256"]


def test_streamed_output_with_host_trace(dataset, golden, tmp_path):
    """A streamed run with the host timeline on (GHOSTM_TRACE=1, read once per
    process, so in a child process): the per-piece trace counters and the
    writer's marks must not disturb the run, and the file is the reference's."""
    import subprocess
    import sys

    d = dataset("syn_small")
    out = tmp_path / "traced.out"
    code = ("import sys; sys.path.insert(0, sys.argv[1]); from ghostm_amd.aligner import Session; "
            "s = Session(['-i', sys.argv[2] + '/q', '-d', sys.argv[2] + '/db', '-o', sys.argv[3], '-D', '0']); "
            "s.run(to_file=True); s.close()")
    env = dict(os.environ, GHOSTM_TRACE="1", GHOSTM_SEGMENT_CANDS="300", GHOSTM_TAIL_CANDS="40")
    r = subprocess.run([sys.executable, "-c", code, cases.REPO, d, str(out)], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "w_end" in r.stderr and "fmt_wall_max_us" in r.stderr
    assert _sha(out.read_bytes()) == golden["aln"]["syn_small/default"]["sha256"]


def test_streamed_output_unwritable_path(dataset, tmp_path):
    """As the reference's unchecked ofstream: an -o path that cannot be opened
    writes nothing and the run still succeeds."""
    d = dataset("syn_small")
    bad = str(tmp_path / "no_such_dir" / "x.out")
    with Session(["-i", os.path.join(d, "q"), "-d", os.path.join(d, "db"), "-o", bad, "-D", "0"]) as s:
        s.run(to_file=True)
        assert len(s.output()) > 0
    assert not os.path.exists(bad)


# ----------------------------------------------------------- full workloads
FULL = os.path.join(cases.GOLDEN, "full_golden.json")


def _full_pins():
    if not os.path.exists(FULL):
        return {}
    with open(FULL) as f:
        return {k: v for k, v in json.load(f).items() if isinstance(v, dict)}


MULTI_BATCH = ["cfg4_20k_l1", "cfg4_20k_l1_b20y2", "dna40k_l1", "dna40k_l1_b20"]


@pytest.mark.parametrize("name", ["cfg2", "cfg3", "cfg5", "cfg4"] + sorted(n for n in workloads.WORKLOADS
                                                                            if n.startswith("cfg5_g"))
                         + MULTI_BATCH)
def test_full_workload_matches_reference(name, tmp_path):
    """The complete BASELINE workload, formatted here and searched by the HIP
    path, against the reference CPU program's full output (sha256, lines)."""
    pin = _full_pins().get(name)
    if pin is None:
        pytest.skip(f"{name} not pinned in full_golden.json")
    db = workloads.make_db(name, str(tmp_path / "db"))
    q = workloads.make_queries(name, str(tmp_path / "q"))
    aln = workloads.WORKLOADS[name]["aln"]
    with Session(["-i", q, "-d", db, "-o", str(tmp_path / "out"), "-D", "0"] + aln) as s:
        s.run()
        text = s.output()
        st = s.stats()
    assert len(text) == pin["bytes"]
    assert text.count(b"\n") == pin["lines"]
    assert _sha(text) == pin["sha256"]
    # a DNA read is searched as its six frames
    frames = 6 if "d" in workloads.WORKLOADS[name]["qry"] else 1
    assert st["queries"] == pin["queries"] * frames


@pytest.mark.parametrize("name,world", [("cfg4", 8), ("cfg3", 3), ("cfg4_20k_l1", 3), ("cfg4_20k_l1", 8),
                                        ("cfg4_20k_l1_b20y2", 8), ("dna40k_l1", 3), ("dna40k_l1_b20", 8)])
def test_full_workload_sharded_matches_reference(name, world, tmp_path):
    """The headline workload as the driver's 8-GPU run cuts it: `world` shard
    sessions (GhostmSessionCreateShard, one after another on this GPU), their
    outputs concatenated in rank order against the reference CPU program's
    full output, and their records against the unsharded run's. The `_l1`
    workloads run several batches (`-l 1`), pinned by ONE reference process:
    every shard replays the unsharded batch cuts."""
    pin = _full_pins().get(name)
    if pin is None:
        pytest.skip(f"{name} not pinned in full_golden.json")
    db = workloads.make_db(name, str(tmp_path / "db"))
    q = workloads.make_queries(name, str(tmp_path / "q"))
    argv = ["-i", q, "-d", db, "-o", str(tmp_path / "out"), "-D", "0"] + workloads.WORKLOADS[name]["aln"]
    h = hashlib.sha256()
    nbytes = 0
    recs = []
    for r in range(world):
        with Session(argv, shard=(r, world)) as s:
            s.run()
            text = s.output()
            h.update(text)
            nbytes += len(text)
            recs.append(s.hits())
    assert nbytes == pin["bytes"]
    assert h.hexdigest() == pin["sha256"]
    with Session(argv) as s:
        s.run()
        assert np.concatenate(recs).tobytes() == s.hits().tobytes()
