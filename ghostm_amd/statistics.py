"""Karlin–Altschul parameters through the C ABI.

Mirrors the reference's Statistics (statistics.cpp:100-112) and BLAST's
BlastComputeLengthAdjustment (karlin.cpp:393-476); the arithmetic lives in
libghostm_hip.so (csrc/karlin_params.cpp).
"""
from __future__ import annotations

import ctypes
from typing import NamedTuple

from . import native


class KarlinParameters(NamedTuple):
    lambda_: float
    K: float
    H: float


def read_score_matrix(path: str) -> list[int]:
    """The 32x32 matrix `aln -M path` uses, row-major (built-in BLOSUM62 when
    the file cannot be opened, score_matrix_reader.cpp:44-113)."""
    lib = native.load()
    buf = (ctypes.c_int * 1024)()
    if lib.GhostmReadScoreMatrix(path.encode(), buf) != 0:
        raise RuntimeError(native.last_error())
    return list(buf)


def ungapped_ideal_karlin(matrix: str | list[int]) -> KarlinParameters:
    """Statistics::CalculateUngappedIdealKarlinParameters for a matrix path or
    a 1024-entry matrix; float32 values bit-identical to the reference's."""
    lib = native.load()
    m = read_score_matrix(matrix) if isinstance(matrix, str) else list(matrix)
    if len(m) != 1024:
        raise ValueError("score matrix must have 32*32 entries")
    arr = (ctypes.c_int * 1024)(*m)
    lam, k, h = ctypes.c_float(), ctypes.c_float(), ctypes.c_float()
    if lib.GhostmKarlinUngapped(arr, ctypes.byref(lam), ctypes.byref(k), ctypes.byref(h)) != 0:
        raise ValueError(native.last_error())
    return KarlinParameters(lam.value, k.value, h.value)


def length_adjustment(K: float, logK: float, alpha_d_lambda: float, beta: float, query_length: int,
                      db_length: int, db_num_seqs: int) -> tuple[int, bool]:
    """BlastComputeLengthAdjustment: (adjustment, converged)."""
    lib = native.load()
    adj = ctypes.c_int()
    rc = lib.GhostmLengthAdjustment(K, logK, alpha_d_lambda, beta, query_length, db_length, db_num_seqs,
                                    ctypes.byref(adj))
    return adj.value, rc == 0
