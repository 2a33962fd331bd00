"""bench.py's all-cores CPU figure: the reference CPU path split
over processes by contiguous query ranges must give the one-process output
byte for byte (queries are independent; names are unique per synthetic query)."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

GHOSTM = os.path.join(REPO, "ghostm_amd", "bin", "ghostm")
CPU_EXES = [os.path.join(REPO, "oracle", "_ref", "ghostm_ref"), os.path.join(REPO, "oracle", "_build", "ghostm_oracle")]


@pytest.mark.skipif(not os.path.exists(GHOSTM) or not any(os.path.exists(p) for p in CPU_EXES),
                    reason="CLI or CPU oracle not built (run __graft_entry__.build())")
@pytest.mark.parametrize("preset,procs", [("cfg2", 1), ("cfg2", 3), ("cfg3", 4)])
def test_cpu_split_matches_one_process(tmp_path, preset, procs):
    import bench
    from ghostm_amd import workloads

    w = str(tmp_path)
    nq = 90
    db = workloads.make_db(preset, os.path.join(w, "db"))
    q = workloads.make_queries(preset, os.path.join(w, "one"), 0, nq)
    exe = next(p for p in CPU_EXES if os.path.exists(p))
    aln = workloads.WORKLOADS[preset]["aln"]
    subprocess.run([exe, "aln", "-i", q, "-d", db, "-o", f"{w}/one.out"] + aln, check=True, capture_output=True)
    one = open(f"{w}/one.out", "rb").read()
    assert one
    joined, dt, nparts, per = bench.reference_split(os.path.join(w, "split"), preset, db, nq, aln, procs)
    assert nparts == procs and dt > 0
    assert joined == one


def test_full_pin_only_for_the_full_workload():
    import bench
    from ghostm_amd import workloads

    pins = bench._json(bench.FULL_GOLDEN) or {}
    for name, w in workloads.WORKLOADS.items():
        if name in pins:
            assert bench.full_pin(name, w["queries"], list(w["aln"])) is not None
        assert bench.full_pin(name, w["queries"] - 1, list(w["aln"])) is None
        assert bench.full_pin(name, w["queries"], list(w["aln"]) + ["-b", "3"]) is None
