"""BASELINE.json workloads as deterministic recipes.

Each recipe names the `ghostm synth` arguments of its query set (every query is a
function of (seed, index), so `-f first -n count` writes exactly a range of the
full set), its DB (generated, or an existing FASTA) and the `qry`/`aln` options.
bench.py builds its inputs from these, tests/golden/make_full_golden.py pins the
reference CPU program's full output for each, and the GPU tests rebuild them to
compare with that pin.
"""
from __future__ import annotations

import os
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
GHOSTM = os.path.join(PKG, "bin", "ghostm")
GOLDEN = os.path.join(REPO, "tests", "golden")
TESTSET_DB = os.path.join(GOLDEN, "testset_db.fasta")
PAM250 = os.path.join(GOLDEN, "matrices", "PAM250")

WORKLOADS = {
    # configs[1] substitute: testset/large_queries.fasta is absent from the reference
    # (.MISSING_LARGE_BLOBS); 100k queries of 20-127 aa sampled from the
    # testset/db.fasta subjects (80 %, 15 % substitutions) or background-random,
    # searched against testset/db.fasta
    "cfg2": {"synth": ["-s", "2", "-a", "20", "-b", "127", "-D", TESTSET_DB], "queries": 100_000,
             "db": ("fasta", TESTSET_DB), "qry": ["-l", "127"], "aln": [],
             "workload": "cfg2 substitute: 100k queries (20-127 aa) sampled from testset/db.fasta subjects "
                         "vs testset/db.fasta"},
    "cfg3": {"synth": ["-s", "3", "-N", "5000000"], "queries": 100_000, "db": ("synth", 5_000_000, 3),
             "qry": ["-l", "300"], "aln": [],
             "workload": "cfg3: synthetic 100k queries (L=127) x 5M-residue DB"},
    "cfg4": {"synth": ["-s", "4", "-N", "10000000"], "queries": 1_000_000, "db": ("synth", 10_000_000, 4),
             "qry": ["-l", "300"], "aln": [],
             "workload": "cfg4: synthetic 1M queries (avg 300 aa requested, L=127) x 10M-residue DB"},
    "cfg5": {"synth": ["-s", "5", "-N", "5000000"], "queries": 100_000, "db": ("synth", 5_000_000, 5),
             "qry": ["-l", "300"], "aln": ["-r", "64", "-M", PAM250, "-y", "2"],
             # the wide band makes the reference ~3x slower per query: smaller CPU samples
             "cpu_sample": 4000, "cpu_sample_all": 8000,
             "workload": "cfg5: wide band -r 64, PAM250 11/1, -y 2; synthetic 100k queries x 5M-residue DB"},
}
# BASELINE configs[4] is a gap-open/extend sweep: the other seven points of
# {8, 10, 11, 14} x {1, 2} on the cfg5 data (G11/E1 is "cfg5" itself)
for _g, _e in ((8, 1), (8, 2), (10, 1), (10, 2), (11, 2), (14, 1), (14, 2)):
    WORKLOADS[f"cfg5_g{_g}e{_e}"] = dict(
        WORKLOADS["cfg5"], aln=["-r", "64", "-M", PAM250, "-G", str(_g), "-E", str(_e), "-y", "2"],
        workload=f"cfg5 gap sweep: -r 64, PAM250 {_g}/{_e}, -y 2; synthetic 100k queries x 5M-residue DB")

# Multi-batch pins: the reference's batch loop (aligner.cpp:131-171,
# 383-391, 511-514) cut by a real `-l 1` (2^20 candidates per batch), run as ONE
# reference process, since the cuts depend on the whole query chunk. The first
# 20k cfg4 queries have ~2.5 M candidates (3 batches); the DNA set's six-frame
# name groups are split by batch cuts.
_CFG4_20K = dict(WORKLOADS["cfg4"], queries=20_000, single_process=True)
WORKLOADS["cfg4_20k_l1"] = dict(_CFG4_20K, aln=["-l", "1"],
                                workload="first 20k cfg4 queries x 10M-residue DB, -l 1 (multi-batch)")
WORKLOADS["cfg4_20k_l1_b20y2"] = dict(_CFG4_20K, aln=["-l", "1", "-b", "20", "-y", "2"],
                                      workload="first 20k cfg4 queries x 10M-residue DB, -l 1 -b 20 -y 2")
_DNA = {"synth": ["-s", "21", "-N", "5000000", "-t", "dna", "-l", "300"], "queries": 40_000,
        "db": ("synth", 5_000_000, 21), "qry": ["-t", "d", "-l", "300"], "single_process": True,
        "cpu_sample": 2000, "cpu_sample_all": 4000}
WORKLOADS["dna40k_l1"] = dict(_DNA, aln=["-l", "1"],
                              workload="40k DNA reads (300 nt, six frames) x 5M-residue DB, -l 1 (multi-batch)")
WORKLOADS["dna40k_l1_b20"] = dict(_DNA, aln=["-l", "1", "-b", "20"],
                                  workload="40k DNA reads (300 nt, six frames) x 5M-residue DB, -l 1 -b 20")


def _run(exe: str, *args: str) -> None:
    subprocess.run([exe, *args], check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)


def make_db(name: str, root: str, exe: str = GHOSTM) -> str:
    """Format the workload's DB under root (formatter `exe`: this repo's `ghostm`,
    or the reference program for the golden pins). Returns the DB prefix."""
    w = WORKLOADS[name]
    os.makedirs(root, exist_ok=True)
    prefix = os.path.join(root, "db")
    if w["db"][0] == "synth":
        _, residues, seed = w["db"]
        _run(GHOSTM, "synth", "-d", f"{root}/db.fa", "-N", str(residues), "-s", str(seed))
        _run(exe, "db", "-i", f"{root}/db.fa", "-o", prefix)
        os.remove(f"{root}/db.fa")
    else:
        _run(exe, "db", "-i", w["db"][1], "-o", prefix)
    return prefix


def make_queries(name: str, root: str, first: int = 0, count: int | None = None, exe: str = GHOSTM) -> str:
    """Format queries [first, first + count) of the workload under root; returns
    the query prefix."""
    w = WORKLOADS[name]
    n = w["queries"] - first if count is None else count
    os.makedirs(root, exist_ok=True)
    _run(GHOSTM, "synth", "-q", f"{root}/q.fa", "-n", str(n), "-f", str(first), *w["synth"])
    _run(exe, "qry", "-i", f"{root}/q.fa", "-o", f"{root}/q", *w["qry"])
    os.remove(f"{root}/q.fa")
    return f"{root}/q"
