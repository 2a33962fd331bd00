"""The CPU oracle (oracle/ghostm_oracle.cpp) against the reference's own fixtures:
the README known-answer table (README.rdoc:138-149), the protein testset and the
golden outputs of the compiled reference CPU path (tests/golden/golden.json)."""
import os

import pytest

import cases

SMALL = [v for v in cases.VARIANTS if v[0] not in cases.SLOW_FOR_ORACLE]


def test_readme_known_answer_matches_readme_table(dataset, tmp_path):
    """README.rdoc:138-149 lists these 12 rows (with query/subject names swapped:
    the README ran the roles the other way round)."""
    d = dataset("readme_kat")
    got = cases.run_aln(cases.ORACLE, d, [], {}, str(tmp_path / "o.out")).decode()
    rows = [line.split("\t") for line in got.splitlines()]
    assert len(rows) == 12
    # README.rdoc:138-149 verbatim (its runs had the words query/subject swapped)
    readme = """\
query0 subject0 100 25 25 1 25 2.75456e-15 60.4622
query0 subject6 100 10 10 16 25 2.58417e-05 27.335
query1 subject0 100 24 24 1 24 1.36707e-14 58.151
query1 subject6 100 9 9 16 24 0.000128251 25.0238
query2 subject5 100 25 25 1 25 4.55093e-10 43.1282
query2 subject6 84.2105 19 16 1 19 1.15998e-05 28.4906
query3 subject6 100 25 25 1 25 2.85052e-12 50.447
query3 subject5 84.2105 19 16 7 25 1.15998e-05 28.4906
query3 subject0 100 10 10 16 25 2.58417e-05 27.335
query4 subject6 100 25 25 1 25 2.85052e-12 50.447
query4 subject5 84.2105 19 16 7 25 1.15998e-05 28.4906
query4 subject0 100 10 10 16 25 2.58417e-05 27.335""".splitlines()
    for ours, theirs in zip(rows, readme):
        t = theirs.split()
        assert ours[0].strip() == t[0].replace("query", "subject")
        assert ours[1].strip() == t[1].replace("subject", "query")
        assert ours[2:9] == t[2:9]
        assert ours[9] == ""  # trailing tab of the default style
    with open(os.path.join(cases.GOLDEN, "readme_kat.out"), "rb") as f:
        assert got.encode() == f.read()


@pytest.mark.parametrize("ds,var,opts,env", SMALL, ids=[f"{v[0]}/{v[1]}" for v in SMALL])
def test_oracle_matches_reference_golden(ds, var, opts, env, dataset, golden, tmp_path):
    d = dataset(ds)
    out = tmp_path / "o.out"
    text = cases.run_aln(cases.ORACLE, d, opts, env, str(out))
    want = golden["aln"][f"{ds}/{var}"]
    assert text.count(b"\n") == want["lines"]
    assert cases.sha256(str(out)) == want["sha256"]


def test_oracle_stage_dump(dataset, tmp_path):
    """The stage dump used by the GPU stage-parity tests is consistent with the
    final output (every printed hit has a traceback record)."""
    d = dataset("syn_small")
    prefix = str(tmp_path / "dump")
    cases.run_aln(cases.ORACLE, d, ["-y", "1"], {"GHOSTM_ORACLE_DUMP": prefix}, str(tmp_path / "o"))
    import numpy as np

    cand = np.fromfile(prefix + ".cand", dtype="<u4").reshape(-1, 4)
    tb = np.fromfile(prefix + ".tb", dtype="<u4").reshape(-1, 5)
    lines = open(tmp_path / "o").read().splitlines()
    assert len(tb) == len(lines)
    assert len(cand) > len(tb)
    # candidates are in (query, start) order
    key = cand[:, 0].astype(np.int64) << 32 | cand[:, 1]
    assert np.all(np.diff(key) > 0)
