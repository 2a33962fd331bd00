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
@pytest.mark.parametrize("procs", [1, 3])
def test_cpu_baseline_all_cores_matches_one_process(tmp_path, procs):
    import bench

    w = str(tmp_path)
    nq, db_res, first = 60, 200_000, 17
    bench.make_data(w, nq, db_res, first, seed=3)
    sub = os.path.join(w, "sample")
    os.makedirs(sub)
    subprocess.run([GHOSTM, "synth", "-q", f"{sub}/q.fa", "-n", str(nq), "-N", str(db_res), "-s", "3",
                    "-f", str(first)], check=True, capture_output=True)
    subprocess.run([GHOSTM, "qry", "-i", f"{sub}/q.fa", "-o", f"{sub}/q", "-l", "300"], check=True,
                   capture_output=True)
    exe = next(p for p in CPU_EXES if os.path.exists(p))
    subprocess.run([exe, "aln", "-i", f"{sub}/q", "-d", f"{w}/db", "-o", f"{sub}/cpu.out"], check=True,
                   capture_output=True)
    assert os.path.getsize(f"{sub}/cpu.out") > 0
    r = bench.cpu_baseline_multi(w, nq, db_res, first, residues=1000, seed=3, aln_args=[], procs=procs)
    assert r is not None and r["cores"] == procs
    assert r["identical_to_one_process"]
