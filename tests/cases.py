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
# the same reference objects linked against libghostm_hip.so (the drop-in), not a trap stub
REF_PLUGIN = os.path.join(REPO, "oracle", "_ref", "ghostm_ref_plugin")
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
    # the cfg4 generator's own DB (10M residues, seed 4) and its first 5000
    # queries: the K1 size classes of the headline workload (97 % class 1,
    # 3 % class 2), its candidate density and the >256-candidate pass
    "syn_scale": [
        ("synth", ["-d", "{d}/db.fa", "-q", "{d}/q.fa", "-n", "5000", "-N", "10000000", "-s", "4"]),
        ("db", ["-i", "{d}/db.fa", "-o", "{d}/db"]),
        ("qry", ["-i", "{d}/q.fa", "-o", "{d}/q", "-l", "300"]),
    ],
    # low-complexity subjects and queries (poly-Q, AKE repeats): K1 class 3
    # (global merge, > 16384 list entries), queries with ~1000 candidates (the
    # offset pass) and name groups of heavily tied scores beyond the K4 wave
    # kernel's LDS capacity (its one-lane fallback), std::sort ties decide subjects
    "syn_repeat": [
        ("synth", ["-d", "{d}/db.fa", "-q", "{d}/q.fa", "-n", "300", "-N", "200000", "-s", "13"]),
        ("py", ["gen_repeat", "{d}"]),
        ("db", ["-i", "{d}/db.fa", "-o", "{d}/db"]),
        ("qry", ["-i", "{d}/q.fa", "-o", "{d}/q", "-l", "300"]),
    ],
    # BASELINE configs[1] substitute at 20 % scale (the full 100k set is pinned in
    # full_golden.json): queries of 20-127 aa sampled from testset/db.fasta
    "cfg2_20k": [
        ("synth", ["-q", "{d}/q.fa", "-n", "20000", "-s", "2", "-a", "20", "-b", "127", "-D",
                   "{golden}/testset_db.fasta"]),
        ("db", ["-i", "{golden}/testset_db.fasta", "-o", "{d}/db"]),
        ("qry", ["-i", "{d}/q.fa", "-o", "{d}/q", "-l", "127"]),
    ],
    # subjects of 10-20 residues: every K2 window crosses up to 15 subject ENDs
    # (the restart-level kernel's levels), and of 4-9 (more ENDs per window than
    # the levels hold: the second-END reset kernel runs instead)
    "syn_subj10": [
        ("synth", ["-d", "{d}/db.fa", "-q", "{d}/q.fa", "-n", "300", "-N", "40000", "-s", "17",
                   "-a", "60", "-b", "127", "-m", "10", "-x", "20"]),
        ("db", ["-i", "{d}/db.fa", "-o", "{d}/db"]),
        ("qry", ["-i", "{d}/q.fa", "-o", "{d}/q", "-l", "127"]),
    ],
    "syn_subj4": [
        ("synth", ["-d", "{d}/db.fa", "-q", "{d}/q.fa", "-n", "300", "-N", "30000", "-s", "19",
                   "-a", "60", "-b", "127", "-m", "4", "-x", "9"]),
        ("db", ["-i", "{d}/db.fa", "-o", "{d}/db"]),
        ("qry", ["-i", "{d}/q.fa", "-o", "{d}/q", "-l", "127"]),
    ],
    # the same queries against a one-subject DB (DB::GetID's early return,
    # reference db.h:115-117, is the only branch taken)
    "cfg2_single": [
        ("synth", ["-q", "{d}/q.fa", "-n", "5000", "-s", "2", "-a", "20", "-b", "127", "-D",
                   "{golden}/testset_db.fasta"]),
        ("py", ["gen_single_subject", "{golden}/testset_db.fasta", "{d}/db.fa"]),
        ("db", ["-i", "{d}/db.fa", "-o", "{d}/db"]),
        ("qry", ["-i", "{d}/q.fa", "-o", "{d}/q", "-l", "127"]),
    ],
}


def gen_repeat(d: str) -> None:
    """Append deterministic low-complexity subjects and queries to a synth
    dataset (syn_repeat)."""
    import random

    r = random.Random(1313)
    aa = "ARNDCQEGHILKMFPSTWYV"

    def mutate(s: str, rate: float) -> str:
        return "".join(aa[r.randrange(20)] if r.random() < rate else ch for ch in s)

    def fasta(name: str, seq: str) -> str:
        return f">{name}\n" + "".join(seq[i:i + 60] + "\n" for i in range(0, len(seq), 60))

    with open(f"{d}/db.fa", "a") as f:
        for i in range(40):
            f.write(fasta(f"polyQ{i}", mutate("Q" * r.randint(300, 600), 0.03)))
        for i in range(20):
            f.write(fasta(f"ake{i}", mutate("AKE" * r.randint(100, 200), 0.03)))
    with open(f"{d}/q.fa", "a") as f:
        for i in range(4):
            f.write(fasta(f"rq{i}", mutate("Q" * r.randint(127, 200), 0.02 * i)))
        for i in range(4):
            f.write(fasta(f"rake{i}", mutate("AKE" * r.randint(43, 70), 0.02 * i)))
        for i in range(6):  # a low-complexity island inside a random query
            left = "".join(r.choice(aa) for _ in range(r.randint(10, 60)))
            right = "".join(r.choice(aa) for _ in range(r.randint(10, 60)))
            f.write(fasta(f"rmix{i}", left + ("Q" if i % 2 else "AKE") * r.randint(4, 12) + right))


def gen_single_subject(src: str, out: str) -> None:
    """The first record of a FASTA file (cfg2_single's one-subject DB)."""
    recs = open(src).read().split(">")[1:]
    with open(out, "w") as f:
        f.write(">" + recs[0])

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
    ("syn_chunks", "b20_y2", ["-b", "20", "-y", "2"], {}),
    ("syn_scale", "default", [], {}),
    ("syn_repeat", "default", [], {}),
    ("syn_repeat", "b20_y2", ["-b", "20", "-y", "2"], {}),
    ("cfg2_20k", "default", [], {}),
    ("cfg2_20k", "y2", ["-y", "2"], {}),
    ("cfg2_single", "default", [], {}),
    ("syn_subj10", "default", [], {}),
    ("syn_subj10", "y2", ["-y", "2"], {}),
    ("syn_subj4", "default", [], {}),
] + [
    # BASELINE configs[4]: -r 64, PAM250, -y 2 over the whole gap sweep
    # {8,10,11,14} x {1,2} (G11/E1 is syn_small/r64_pam250 above)
    ("syn_small", f"r64_pam250_g{g}e{e}", ["-r", "64", "-M", PAM250, "-G", str(g), "-E", str(e), "-y", "2"], {})
    for g in (8, 10, 11, 14) for e in (1, 2) if (g, e) != (11, 1)
]

# variants whose oracle run takes more than a few seconds: GPU tests only (their
# golden values come from the reference program itself)
SLOW_FOR_ORACLE = {"syn_chunks", "syn_scale", "cfg2_20k"}

# batch-cut cases (-l in candidates via the test hook); oracle-checked only
BATCH_VARIANTS = [
    ("syn_small", "cut50", [], {"GHOSTM_MAX_LIST_OVERRIDE": "50"}),
    ("syn_small", "cut1", [], {"GHOSTM_MAX_LIST_OVERRIDE": "1"}),
    ("syn_small", "cut700", [], {"GHOSTM_MAX_LIST_OVERRIDE": "700"}),
    ("syn_dna", "cut100", [], {"GHOSTM_MAX_LIST_OVERRIDE": "100"}),
    ("syn_dna", "cut13", ["-y", "2"], {"GHOSTM_MAX_LIST_OVERRIDE": "13"}),
    # -b above std::sort's insertion threshold (16): the carried result lists are
    # re-sorted by introsort every batch, so tie order matters across batches
    ("syn_small", "cut300_b20", ["-b", "20", "-y", "2"], {"GHOSTM_MAX_LIST_OVERRIDE": "300"}),
    ("syn_repeat", "cut2000_b20", ["-b", "20"], {"GHOSTM_MAX_LIST_OVERRIDE": "2000"}),
    ("syn_dna", "cut57_b3", ["-b", "3"], {"GHOSTM_MAX_LIST_OVERRIDE": "57"}),
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
        if tool == "py":
            globals()[a[0]](*a[1:])
        else:
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


def k1_list_entries(d: str, qprefix: str = "q", dprefix: str = "db", shift: int = 2) -> "np.ndarray":
    """Per query of chunk 0: the number of K1 list entries (positions p >= j*shift
    over the query's seed lists j), which picks the K1 size class
    (ghostm_amd/csrc/device.hip SeedCaps). Numpy restatement of the list
    selection of SearchNextCpu (reference aligner.cpp:399-430), for the tests
    that assert every class runs."""
    import numpy as np

    inf = np.fromfile(f"{d}/{qprefix}_0.inf", dtype="<u4")
    nq, L = int(inf[0]), int(inf[1])
    q = np.fromfile(f"{d}/{qprefix}_0.seq", dtype=np.uint8)[: nq * L].reshape(nq, L).astype(np.int64)
    raw = np.fromfile(f"{d}/{dprefix}_0.ind", dtype="<u4")
    seed, kcl, npos = (int(x) for x in raw[:3])
    kc = raw[3:3 + kcl].astype(np.int64)
    pos = raw[3 + kcl:3 + kcl + npos].astype(np.int64)
    offs = [t for t in range(32) if (seed >> t) & 1]
    span = max(offs) + 1
    nl = (L - span) // shift + 1
    out = np.zeros(nq, dtype=np.int64)
    for j in range(nl):
        key = np.zeros(nq, dtype=np.int64)
        for t in offs:
            key = (key << 5) | q[:, j * shift + t]
        b, e = kc[key], kc[key + 1]
        # positions before the list's diagonal origin j*shift are skipped
        lo = np.array([bb + np.searchsorted(pos[bb:ee], j * shift) if ee > bb else bb for bb, ee in zip(b, e)])
        out += e - lo
    return out
