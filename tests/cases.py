"""Shared test datasets and option variants.

Every dataset is produced from committed FASTA (the reference testset) or from
`ghostm synth` (deterministic) and formatted with this repo's `ghostm db|qry`,
whose files are pinned byte-for-byte to the reference formatters by the hashes in
golden/golden.json. Expected `aln` outputs come from the reference CPU program
(oracle/_ref) via golden/make_golden.py, and are re-checked live against the
oracle restatement.
"""
from __future__ import annotations

import hashlib
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLDEN = os.path.join(HERE, "golden")
GHOSTM = os.path.join(REPO, "ghostm_amd", "bin", "ghostm")
ORACLE = os.path.join(REPO, "oracle", "_build", "ghostm_oracle")
REF = os.path.join(REPO, "oracle", "_ref", "ghostm_ref")
PAM250 = os.path.join(GOLDEN, "matrices", "PAM250")
PAM30 = os.path.join(GOLDEN, "matrices", "pam30_name", "PAM30")

# name -> list of (tool, args); {d} = dataset dir. Tools: synth | db | qry
DATASETS = {
    "readme_kat": [
        ("qry", ["-t", "d", "-i", "{golden}/testset_db.fasta", "-o", "{d}/q"]),
        ("db", ["-i", "{golden}/testset_queries.fasta", "-o", "{d}/db"]),
    ],
    "protein_testset": [
        ("qry", ["-i", "{golden}/testset_queries.fasta", "-o", "{d}/q"]),
        ("db", ["-i", "{golden}/testset_db.fasta", "-o", "{d}/db"]),
    ],
    "syn_small": [
        ("synth", ["-d", "{d}/db.fa", "-q", "{d}/q.fa", "-n", "400", "-N", "200000", "-s", "7"]),
        ("db", ["-i", "{d}/db.fa", "-o", "{d}/db"]),
        ("qry", ["-i", "{d}/q.fa", "-o", "{d}/q", "-l", "300"]),
    ],
    "syn_dna": [
        ("synth", ["-d", "{d}/db.fa", "-q", "{d}/q.fa", "-n", "300", "-N", "150000", "-s", "5",
                   "-t", "dna", "-l", "150"]),
        ("db", ["-i", "{d}/db.fa", "-o", "{d}/db"]),
        ("qry", ["-i", "{d}/q.fa", "-o", "{d}/q", "-t", "d", "-l", "150"]),
    ],
    "syn_short": [  # short queries (L=40, three lanes per candidate) and k=3 seeds
        ("synth", ["-d", "{d}/db.fa", "-q", "{d}/q.fa", "-n", "500", "-N", "100000", "-s", "9",
                   "-a", "20", "-b", "60", "-m", "3", "-x", "300"]),
        ("db", ["-i", "{d}/db.fa", "-o", "{d}/db", "-k", "3"]),
        ("qry", ["-i", "{d}/q.fa", "-o", "{d}/q", "-l", "40"]),
    ],
    "syn_chunks": [  # 2 query chunks x 3 DB chunks
        ("synth", ["-d", "{d}/db.fa", "-q", "{d}/q.fa", "-n", "7000", "-N", "2800000", "-s", "11"]),
        ("db", ["-i", "{d}/db.fa", "-o", "{d}/db", "-l", "1"]),
        ("qry", ["-i", "{d}/q.fa", "-o", "{d}/q", "-l", "300", "-L", "1"]),
    ],
}

# (dataset, variant name, aln option list, env)
VARIANTS = [
    ("readme_kat", "default", [], {}),
    ("readme_kat", "y2", ["-y", "2"], {}),
    ("protein_testset", "y0", [], {}),
    ("protein_testset", "y1", ["-y", "1"], {}),
    ("protein_testset", "y2", ["-y", "2"], {}),
    ("syn_small", "default", [], {}),
    ("syn_small", "y1", ["-y", "1"], {}),
    ("syn_small", "y2", ["-y", "2"], {}),
    ("syn_small", "b3", ["-b", "3"], {}),
    ("syn_small", "b20_t1", ["-b", "20", "-t", "1", "-y", "2"], {}),
    ("syn_small", "t0", ["-t", "0"], {}),
    ("syn_small", "t3", ["-t", "3"], {}),
    ("syn_small", "s1", ["-s", "1"], {}),
    ("syn_small", "s3", ["-s", "3"], {}),
    ("syn_small", "r4", ["-r", "4"], {}),
    ("syn_small", "r64_pam250", ["-r", "64", "-M", PAM250, "-y", "2"], {}),
    ("syn_small", "pam250_g8e1", ["-M", PAM250, "-G", "8", "-E", "1", "-y", "2"], {}),
    ("syn_small", "pam250_g14e2", ["-M", PAM250, "-G", "14", "-E", "2", "-y", "2"], {}),
    ("syn_small", "pam30_name", ["-M", PAM30, "-G", "9", "-E", "1"], {}),
    ("syn_small", "e0", ["-e", "0"], {}),
    ("syn_small", "e6", ["-e", "6"], {}),
    ("syn_small", "l0", ["-l", "0"], {}),
    ("syn_small", "g0e0", ["-G", "0", "-E", "0", "-y", "2"], {}),
    ("syn_dna", "default", [], {}),
    ("syn_dna", "b5_y2", ["-b", "5", "-y", "2"], {}),
    ("syn_short", "default", [], {}),
    ("syn_short", "t1_y2", ["-t", "1", "-y", "2"], {}),
    ("syn_chunks", "default", [], {}),
    ("syn_chunks", "S1", ["-S", "1"], {}),
    ("syn_chunks", "L0", ["-L", "0"], {}),
]

# batch-cut cases (-l in candidates via the test hook); oracle-checked only
BATCH_VARIANTS = [
    ("syn_small", "cut50", [], {"GHOSTM_MAX_LIST_OVERRIDE": "50"}),
    ("syn_small", "cut1", [], {"GHOSTM_MAX_LIST_OVERRIDE": "1"}),
    ("syn_small", "cut700", [], {"GHOSTM_MAX_LIST_OVERRIDE": "700"}),
    ("syn_dna", "cut100", [], {"GHOSTM_MAX_LIST_OVERRIDE": "100"}),
    ("syn_dna", "cut13", ["-y", "2"], {"GHOSTM_MAX_LIST_OVERRIDE": "13"}),
]


def sha256(path: str) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(1 << 20), b""):
            h.update(b)
    return h.hexdigest()


def build_dataset(name: str, root: str) -> str:
    """Create dataset `name` under root/name (cached); returns the directory."""
    d = os.path.join(root, name)
    stamp = os.path.join(d, ".done")
    if os.path.exists(stamp):
        return d
    os.makedirs(d, exist_ok=True)
    for tool, args in DATASETS[name]:
        a = [x.format(d=d, golden=GOLDEN) for x in args]
        subprocess.run([GHOSTM, tool] + a, check=True, capture_output=True)
    open(stamp, "w").close()
    return d


def formatted_files(d: str) -> list[str]:
    """Formatted files of a dataset (what `aln` reads), sorted, relative to d."""
    out = []
    for f in sorted(os.listdir(d)):
        if f.endswith((".inf", ".nam", ".seq", ".pos", ".ind")):
            out.append(f)
    return out


def run_aln(exe: str, d: str, opts: list[str], env: dict, out: str) -> bytes:
    e = dict(os.environ)
    e.update(env)
    subprocess.run([exe, "aln", "-i", os.path.join(d, "q"), "-d", os.path.join(d, "db"),
                    "-o", out] + list(opts), check=True, env=e, capture_output=True)
    with open(out, "rb") as f:
        return f.read()


def parse_ncbi_matrix(path: str):
    """32x32 int32 M[db*32 + query] with the reference reader's rules
    (score_matrix_reader.cpp:73-113)."""
    import numpy as np

    codes = {c: i for i, c in enumerate("ARNDCQEGHILKMFPSTWYVBJZX*")}
    code = lambda ch: codes.get(ch.upper(), 23)  # noqa: E731
    m = np.zeros(32 * 32, dtype=np.int32)
    head, rows = [], []
    n = 0
    for line in open(path).read().split("\n"):
        if not line or line[0] == "#" or n >= 25:
            continue
        f = [x for x in line.split(" ") if x][:25]
        if n == 0:
            head = [x[0] for x in f]
        else:
            r = f[0][0]
            for i, v in enumerate(f[1:], start=1):
                m[code(r) * 32 + code(head[i - 1])] = int(v)
        n += 1
    return m
