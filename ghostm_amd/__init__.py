"""ghostm_amd — MI355X (gfx950) build of the GHOSTM 2.0 `aln` hot path.

Seed lookup, Gotoh score DP and traceback are hand-written HIP kernels in
csrc/; the merge/E-value host logic and the C ABI live in libghostm_hip.so.
"""
from .aligner import Aligner, GhostmError, HIT_DTYPE, Session, format_db, format_queries, run_cli, synth
from .native import BIN_PATH, LIB_PATH, NativeLibraryMissing, load

__all__ = [
    "Aligner",
    "Session",
    "GhostmError",
    "HIT_DTYPE",
    "format_db",
    "format_queries",
    "synth",
    "run_cli",
    "load",
    "LIB_PATH",
    "BIN_PATH",
    "NativeLibraryMissing",
]
