"""GPU vs CPU k-mer index build for the `db` formatter on the
BASELINE cfg4 database (synthetic 10M residues, splitmix64 seed 4, -k 4).

Prints one JSON line: the device time of GhostmBuildIndexGpu (HIP events, upload
excluded; best of --reps), its algorithmic-byte rate against HBM peak (bytes =
the .seq read + keys_count and positions written), the wall time of `ghostm db`
with and without -D 0, and whether the two .ind files are identical.

    python tools/bench_index.py [--db-residues 10000000] [--reps 5]
"""
from __future__ import annotations

import argparse
import ctypes
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def sha(p: str) -> str:
    with open(p, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def main() -> None:
    import numpy as np

    from ghostm_amd.native import BIN_PATH, last_error, load

    ap = argparse.ArgumentParser()
    ap.add_argument("--db-residues", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    with tempfile.TemporaryDirectory() as tmp:
        subprocess.run([BIN_PATH, "synth", "-d", f"{tmp}/db.fa", "-q", f"{tmp}/q.fa", "-n", "1",
                        "-N", str(args.db_residues), "-s", "4"], check=True, capture_output=True)
        t0 = time.perf_counter()
        subprocess.run([BIN_PATH, "db", "-i", f"{tmp}/db.fa", "-o", f"{tmp}/cpu"], check=True, capture_output=True)
        cpu_s = time.perf_counter() - t0
        t0 = time.perf_counter()
        subprocess.run([BIN_PATH, "db", "-i", f"{tmp}/db.fa", "-o", f"{tmp}/gpu", "-D", "0"], check=True,
                       capture_output=True)
        gpu_s = time.perf_counter() - t0
        same = sha(f"{tmp}/cpu_0.ind") == sha(f"{tmp}/gpu_0.ind")
        seq = np.fromfile(f"{tmp}/cpu_0.seq", dtype=np.uint8)
        lib = load()
        kcl = 32 ** 4 + 1
        kc = np.zeros(kcl, dtype=np.uint32)
        pos = np.zeros(len(seq), dtype=np.uint32)
        npos = ctypes.c_uint32(0)
        u32 = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))  # noqa: E731
        times = []
        for _ in range(args.reps):
            ms = ctypes.c_float(0)
            rc = lib.GhostmBuildIndexGpu(seq.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), len(seq), 15, kcl,
                                         u32(kc), u32(pos), ctypes.byref(npos), 0, ctypes.byref(ms))
            if rc:
                raise RuntimeError(last_error())
            times.append(ms.value)
        dev_ms = min(times)
        algo = len(seq) + 4 * kcl + 4 * npos.value
        gbs = algo / (dev_ms * 1e-3) / 1e9
        print(json.dumps({
            "component": "db k-mer index build (db_creator.cpp:167-241), GhostmBuildIndexGpu",
            "db_residues": args.db_residues, "seq_bytes": int(len(seq)), "npos": npos.value,
            "device_ms": dev_ms, "device_ms_all": times,
            "roofline": {"bound": "hbm", "achieved": gbs, "peak": 8000.0, "unit": "GB/s", "frac": gbs / 8000.0,
                         "algorithmic_bytes": algo},
            "db_wall_s_cpu_formatter": cpu_s, "db_wall_s_gpu_index": gpu_s,
            "ind_identical": same,
        }), flush=True)


if __name__ == "__main__":
    main()
