"""General Karlin–Altschul parameters against the reference.

tests/golden/karlin_golden.json holds the float32 bits that the reference's own
Statistics::CalculateUngappedIdealKarlinParameters and BlastComputeLengthAdjustment
(statistics.cpp:100-112, karlin.cpp:16-476, compiled from /root/reference by
oracle/Makefile; generator tests/golden/make_karlin_golden.py) printed. The
product's restatement (csrc/karlin_params.cpp) must give the same bits.
"""
from __future__ import annotations

import json
import os
import struct

import numpy as np
import pytest

from ghostm_amd import statistics

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLDEN = json.load(open(os.path.join(HERE, "golden", "karlin_golden.json")))["cases"]


def bits(x: float) -> int:
    return struct.unpack("<I", struct.pack("<f", x))[0]


def as_float(u: int) -> float:
    return struct.unpack("<f", struct.pack("<I", u))[0]


def resolve(path: str) -> str:
    return path if os.path.isabs(path) else os.path.join(REPO, path)


@pytest.mark.parametrize("case", GOLDEN, ids=[os.path.basename(c["path"]) for c in GOLDEN])
def test_ungapped_params_bit_identical(case):
    p = statistics.ungapped_ideal_karlin(resolve(case["path"]))
    assert (bits(p.lambda_), bits(p.K), bits(p.H)) == (case["lambda"], case["K"], case["H"])


@pytest.mark.parametrize("case", [c for c in GOLDEN if c["adjust"]],
                         ids=[os.path.basename(c["path"]) for c in GOLDEN if c["adjust"]])
def test_length_adjustment(case):
    K, H, logK = as_float(case["K"]), as_float(case["H"]), as_float(case["logK"])
    alpha = float(np.float32(1.0) / np.float32(H))  # 1.0f / H in float, as karlin_ref's caller
    for m, n, N, adj, rc in case["adjust"]:
        got, converged = statistics.length_adjustment(K, logK, alpha, 0.0, m, n, N)
        assert (got, 0 if converged else 1) == (adj, rc), (m, n, N)


def test_matrix_reader_matches_builtin_fallback():
    """A path that cannot be opened reads as the built-in BLOSUM62 (reader :50-66)."""
    assert statistics.read_score_matrix("/nonexistent/x") == statistics.read_score_matrix(
        os.path.join(HERE, "golden", "matrices", "BLOSUM62"))


def test_bad_matrix_length():
    with pytest.raises(ValueError):
        statistics.ungapped_ideal_karlin([0] * 10)
