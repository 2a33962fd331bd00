"""ctypes binding of the C ABI in include/ghostm_hip.h (libghostm_hip.so).

The library is built in-tree (ghostm_amd/lib) by `__graft_entry__.build()` /
`make -C ghostm_amd/csrc`. There is no fallback: if the library is missing or a
symbol is absent, loading raises, so nothing silently runs on the CPU.
"""
from __future__ import annotations

import ctypes
import os
import re
from ctypes import POINTER, c_char_p, c_float, c_int, c_size_t, c_uint32, c_uint64, c_void_p

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
# GHOSTM_LIB_PATH selects another build of the same library (A/B timing runs)
LIB_PATH = os.environ.get("GHOSTM_LIB_PATH") or os.path.join(PKG_DIR, "lib", "libghostm_hip.so")
BIN_PATH = os.path.join(PKG_DIR, "bin", "ghostm")
HEADER_PATH = os.path.join(REPO_DIR, "include", "ghostm_hip.h")

u32p = POINTER(c_uint32)

# GhostmAllGatherFn (include/ghostm_hip.h): int (*)(void *ctx, const void *send,
# uint64_t send_bytes, void *recv, const uint64_t *recv_bytes)
ALLGATHER_FN = ctypes.CFUNCTYPE(c_int, c_void_p, c_void_p, c_uint64, c_void_p, POINTER(c_uint64))


class GhostmHit(ctypes.Structure):
    """reference Alignment fields gathered per hit (alignment.h:136-145)."""

    _fields_ = [
        ("query_id", c_uint32),
        ("db_id", c_uint32),
        ("score", c_uint32),
        ("db_start", c_uint32),
        ("db_end", c_uint32),
        ("aln_len", c_uint32),
        ("aln_match", c_uint32),
        ("seq_id", c_float),
    ]


class GhostmStats(ctypes.Structure):
    _fields_ = [
        ("seconds_total", ctypes.c_double),
        ("seconds_seed", ctypes.c_double),
        ("seconds_score", ctypes.c_double),
        ("seconds_traceback", ctypes.c_double),
        ("seconds_merge", ctypes.c_double),
        ("seconds_output", ctypes.c_double),
        ("queries", c_uint64),
        ("query_residues", c_uint64),
        ("candidates", c_uint64),
        ("score_cells", c_uint64),
        ("tracebacks", c_uint64),
        ("traceback_cells", c_uint64),
        ("hits", c_uint64),
        ("batches", c_uint64),
        ("score_launches", c_uint64),
        ("seed_bytes", c_uint64),
        ("score_launches_packed", c_uint64),
        ("score_launches_half", c_uint64),
        ("traceback_launches", c_uint64),
        ("traceback_launches_key", c_uint64),
        ("seed_runs_hash", c_uint64),
        ("score_rechecks", c_uint64),
        ("traceback_launches_scan", c_uint64),
        ("traceback_scan_cells", c_uint64),
        ("merge_launches", c_uint64),
        ("merge_launches_wave", c_uint64),
        ("score_launches_framed", c_uint64),
        ("seed_queries_class", c_uint64 * 4),
        ("seed_queries_wide", c_uint64),
        ("segments", c_uint64),
        ("seed_runs_filter", c_uint64),
        ("seed_filter_overflows", c_uint64),
        ("score_launches_swar", c_uint64),
        ("traceback_launches_scan_swar", c_uint64),
        ("seed_list_entries", c_uint64),
        ("score_launches_unit", c_uint64),
        ("traceback_launches_strips", c_uint64),
        ("seconds_traceback_scan", ctypes.c_double),
        ("score_launches_pair", c_uint64),
        ("seed_table_full", c_uint64),
        ("seed_compact_redo", c_uint64),
        ("score_launches_sparse", c_uint64),
        ("traceback_launches_keyframe", c_uint64),
        ("score_launches_levels", c_uint64),
    ]

    def as_dict(self) -> dict:
        out = {}
        for name, _ in self._fields_:
            v = getattr(self, name)
            if name == "seed_queries_class":
                for k in range(4):
                    out[f"seed_queries_class{k}"] = v[k]
            else:
                out[name] = v
        return out


# name -> (restype, argtypes); covers every function declared in the header
SIGNATURES = {
    "InitGpu": (c_int, []),
    "GetNeededGPUMemorySize": (c_size_t, [c_uint32] * 6),
    "CheckGpuMemory": (c_int, [c_uint32] * 6),
    "SetOptionGpu": (c_int, [c_uint32, POINTER(c_int), c_int]),
    "printGpuInfo": (None, [c_int]),
    "SetQueryGpu": (c_int, [POINTER(ctypes.c_uint8), c_uint32, c_uint32]),
    "SetDbGpu": (c_int, [POINTER(ctypes.c_uint8), c_uint32, u32p, c_uint32, u32p, c_uint32]),
    "SearchNextGpu": (c_uint32, [c_uint32] * 8 + [u32p, u32p]),
    "CalculateScoreGpu": (None, [c_uint32, c_uint32, c_uint32, u32p, u32p, c_uint32, c_uint32, c_int, c_int]),
    "FreeGpu": (c_int, []),
    "GhostmGetLastError": (c_char_p, []),
    "GhostmBuildInfo": (c_char_p, []),
    "GhostmDevicePoolTrim": (c_uint64, []),
    "GhostmDevicePoolInfo": (c_int, [POINTER(c_uint64), POINTER(c_uint64)]),
    "CountCandidatesGpu": (c_int, [c_uint32] * 6 + [u32p]),
    "TraceBackGpu": (c_int, [c_uint32, u32p, u32p, c_uint32, c_uint32, c_int, c_int, u32p, u32p, u32p, POINTER(c_float)]),
    "GhostmBuildIndexGpu": (c_int, [POINTER(ctypes.c_uint8), c_uint32, c_uint32, c_uint32, u32p, u32p, u32p, c_int,
                                    POINTER(c_float)]),
    "GhostmFormatQueriesGpu": (c_int, [POINTER(ctypes.c_uint8), c_uint64, POINTER(c_uint64), u32p, c_uint32, c_uint32,
                                       c_uint32, POINTER(ctypes.c_uint8), c_int, POINTER(c_float)]),
    "GhostmKarlinUngapped": (c_int, [POINTER(c_int), POINTER(c_float), POINTER(c_float), POINTER(c_float)]),
    "GhostmReadScoreMatrix": (c_int, [c_char_p, POINTER(c_int)]),
    "GhostmLengthAdjustment": (c_int, [c_float, c_float, c_float, c_float, c_int, c_uint32, c_int, POINTER(c_int)]),
    "GhostmSessionCreate": (c_void_p, [c_int, POINTER(c_char_p)]),
    "GhostmSessionCreateShard": (c_void_p, [c_int, POINTER(c_char_p), c_int, c_int]),
    "GhostmSessionCreateShardEx": (c_void_p, [c_int, POINTER(c_char_p), c_int, c_int, c_void_p, c_void_p]),
    "GhostmSessionShardRange": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64)]),
    "GhostmSessionHitCapacity": (c_uint64, [c_void_p]),
    "GhostmShardCuts": (c_int, [c_uint64, u32p, POINTER(ctypes.c_uint8), c_int, POINTER(c_uint64)]),
    "GhostmSessionRun": (c_int, [c_void_p]),
    "GhostmSessionRunToFile": (c_int, [c_void_p]),
    "GhostmSessionOutput": (c_size_t, [c_void_p, c_char_p, c_size_t]),
    "GhostmSessionWrite": (c_int, [c_void_p]),
    "GhostmSessionHits": (c_size_t, [c_void_p, POINTER(GhostmHit), c_size_t]),
    "GhostmSessionDeviceHits": (c_size_t, [c_void_p, c_void_p, c_size_t]),
    "GhostmSessionStats": (c_int, [c_void_p, POINTER(GhostmStats)]),
    "GhostmSessionStatsSized": (c_size_t, [c_void_p, POINTER(GhostmStats), c_size_t]),
    "GhostmSessionDestroy": (None, [c_void_p]),
    "GhostmAlignMain": (c_int, [c_int, POINTER(c_char_p)]),
}

_lib = None


class NativeLibraryMissing(RuntimeError):
    pass


def header_functions(path: str = HEADER_PATH) -> list[str]:
    """Function names declared in include/ghostm_hip.h."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"\btypedef\b[^;]*;", "", text)  # function-pointer types are not exports
    names = re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\(", text)
    skip = {"if", "defined", "sizeof"}
    out = []
    for n in names:
        if n in skip or n in out:
            continue
        out.append(n)
    return out


def load() -> ctypes.CDLL:
    """Load libghostm_hip.so (raises NativeLibraryMissing if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryMissing(
            f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
        )
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)  # AttributeError if the symbol is missing
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def device_pool_info() -> tuple[int, int]:
    """(cached bytes, allocations retried after emptying the cache)."""
    cached, retries = c_uint64(0), c_uint64(0)
    load().GhostmDevicePoolInfo(ctypes.byref(cached), ctypes.byref(retries))
    return cached.value, retries.value


def last_error() -> str:
    return (load().GhostmGetLastError() or b"").decode(errors="replace")


def argv_array(args: list[str]):
    arr = (c_char_p * (len(args) + 1))()
    for i, a in enumerate(args):
        arr[i] = a.encode()
    arr[len(args)] = None
    return arr
