"""Pin the general Karlin–Altschul routines to the reference.

Writes a few derived matrix files under tests/golden/matrices/karlin/ (each one
drives a distinct branch of karlin.cpp: the +-1 shortcut of BlastKarlinLHtoK,
a score lattice with gcd 2 and 3, a wide score range, a positive-drift matrix
with no positive root, a matrix without positive scores that BlastScoreChk
rejects), runs oracle/_ref/karlin_ref (the reference's own statistics.cpp and
karlin.cpp, compiled by oracle/Makefile) over them and the committed matrices,
and writes tests/golden/karlin_golden.json: float32 bits of lambda, K, H and
logf(K) plus BlastComputeLengthAdjustment results for fixed (m, n, N).

Runs ONLY in the build container (needs /root/reference):
    make -C oracle ref && python tests/golden/make_karlin_golden.py
"""
from __future__ import annotations

import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
MATRICES = os.path.join(HERE, "matrices")
OUT_DIR = os.path.join(MATRICES, "karlin")
LETTERS = "ARNDCQEGHILKMFPSTWYVBZX*"


def read_rows(path: str) -> list[list[int]]:
    rows = []
    with open(path) as f:
        for line in f:
            if not line.strip() or line.startswith("#") or line.split()[0] == "A" and len(line.split()) == 24:
                continue
            rows.append([int(v) for v in line.split()[1:25]])
    assert len(rows) == 24, path
    return rows


def write_matrix(name: str, rows: list[list[int]], note: str) -> str:
    path = os.path.join(OUT_DIR, name)
    with open(path, "w") as f:
        f.write(f"#  {note}\n")
        f.write("   " + "  ".join(LETTERS) + "\n")
        for a, row in zip(LETTERS, rows):
            f.write(a + " " + " ".join(f"{v:3d}" for v in row) + "\n")
    return path


def derived() -> list[str]:
    os.makedirs(OUT_DIR, exist_ok=True)
    b62 = read_rows(os.path.join(MATRICES, "BLOSUM62"))
    n = len(LETTERS)
    ident = [[1 if i == j else -1 for j in range(n)] for i in range(n)]
    drift = [[2 if i == j else 1 for j in range(n)] for i in range(n)]
    drift[23][23] = -1
    nonpos = [[0 if i == j else -2 for j in range(n)] for i in range(n)]
    return [
        write_matrix("B62x2", [[2 * v for v in r] for r in b62], "BLOSUM62 doubled: score lattice gcd 2"),
        write_matrix("B62x3m", [[3 * v - (1 if v < 0 else 0) for v in r] for r in b62], "BLOSUM62 x3, negatives minus 1"),
        write_matrix("B62x25", [[25 * v for v in r] for r in b62], "BLOSUM62 x25: wide score range"),
        write_matrix("IDENT1", ident, "+1 match / -1 mismatch: the low == -1 shortcut"),
        write_matrix("DRIFT", drift, "positive expected score: no positive lambda"),
        write_matrix("NONPOS", nonpos, "no positive score: rejected by BlastScoreChk"),
    ]


def main() -> None:
    exe = os.path.join(REPO, "oracle", "_ref", "karlin_ref")
    paths = [os.path.join(MATRICES, "BLOSUM62"), os.path.join(MATRICES, "PAM250"),
             os.path.join(MATRICES, "pam30_name", "PAM30")] + derived() + ["/nonexistent/matrix"]
    out = subprocess.run([exe, *paths], check=True, capture_output=True, text=True).stdout
    cases = json.loads(out)
    for c in cases:  # repo-relative paths so the fixture travels
        if c["path"].startswith(REPO):
            c["path"] = os.path.relpath(c["path"], REPO)
    with open(os.path.join(HERE, "karlin_golden.json"), "w") as f:
        json.dump({"generator": "oracle/_ref/karlin_ref (reference statistics.cpp + karlin.cpp)",
                   "cases": cases}, f, indent=1)
        f.write("\n")
    print(f"{len(cases)} cases")


if __name__ == "__main__":
    main()
