"""GPU vs CPU `qry` formatter on the BASELINE cfg4 query set
(1M synthetic protein queries, `qry -l 300` -> width 127) and on a DNA read set
(`qry -t d`, six frames per read).

Prints one JSON line per case: the device time of GhostmFormatQueriesGpu (HIP
events, upload excluded; best of --reps) with its algorithmic bytes (letters
read + records written + 12 B of offsets/lengths per record) against HBM peak,
the wall time of `ghostm qry` with and without -D 0, and whether their files are
identical.

    python tools/bench_qry.py [--queries 1000000] [--reads 200000] [--reps 5]
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
PEAK_HBM_GBS = 8000.0


def sha(p: str) -> str:
    h = hashlib.sha256()
    with open(p, "rb") as f:
        for blk in iter(lambda: f.read(1 << 24), b""):
            h.update(blk)
    return h.hexdigest()


def letters(fa: str):
    """The FASTA's records as (concatenated letters, offsets, lengths), the
    buffer the formatter hands to the device (one chunk)."""
    import numpy as np

    with open(fa, "rb") as f:
        data = f.read()
    seqs = [rec.split(b"\n", 1)[1].replace(b"\n", b"") if b"\n" in rec else b""
            for rec in data.lstrip(b">").split(b"\n>")]
    lens = np.array([len(s) for s in seqs], dtype=np.uint32)
    offs = np.zeros(len(seqs), dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    return np.frombuffer(b"".join(seqs), dtype=np.uint8), offs, lens


def case(tmp: str, name: str, fa: str, opts: list, width: int, dna: bool, reps: int) -> dict:
    import numpy as np

    from ghostm_amd.native import BIN_PATH, last_error, load

    t0 = time.perf_counter()
    subprocess.run([BIN_PATH, "qry", "-i", fa, "-o", f"{tmp}/{name}_cpu"] + opts, check=True, capture_output=True)
    cpu_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    subprocess.run([BIN_PATH, "qry", "-i", fa, "-o", f"{tmp}/{name}_gpu", "-D", "0"] + opts, check=True,
                   capture_output=True)
    gpu_s = time.perf_counter() - t0
    files = sorted(f[len(name) + 4:] for f in os.listdir(tmp) if f.startswith(f"{name}_cpu"))
    same = all(sha(f"{tmp}/{name}_cpu{f}") == sha(f"{tmp}/{name}_gpu{f}") for f in files)
    raw, offs, lens = letters(fa)
    n = len(lens)
    dna_len = max(int(lens[0]), 1) if dna else 0  # the chunk's first read sets the length
    nout = n * (6 if dna_len else 1)
    out = np.zeros(nout * width, dtype=np.uint8)
    lib = load()
    ms = ctypes.c_float(0)
    best = None
    for _ in range(reps):
        rc = lib.GhostmFormatQueriesGpu(raw.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), len(raw),
                                        offs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                        lens.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), n, width, dna_len,
                                        out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), 0, ctypes.byref(ms))
        if rc:
            raise SystemExit(last_error())
        best = ms.value if best is None else min(best, ms.value)
    # algorithmic bytes: the letters the kernel reads, the records it writes,
    # 12 B of (offset, length) per record
    read = int(np.minimum(lens, dna_len if dna_len else width).sum())
    bytes_ = read + nout * width + 12 * n
    return {"case": name, "records_in": n, "records_out": nout, "width": width,
            "device_ms": best, "algorithmic_bytes": bytes_,
            "achieved_gbs": bytes_ / (best * 1e-3) / 1e9 if best else None,
            "hbm_frac": bytes_ / (best * 1e-3) / 1e9 / PEAK_HBM_GBS if best else None,
            "cpu_formatter_s": cpu_s, "gpu_formatter_s": gpu_s, "files_identical": same}


def main() -> None:
    from ghostm_amd.native import BIN_PATH

    ap = argparse.ArgumentParser()
    ap.add_argument("--queries", type=int, default=1_000_000)
    ap.add_argument("--reads", type=int, default=200_000)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    with tempfile.TemporaryDirectory() as tmp:
        subprocess.run([BIN_PATH, "synth", "-q", f"{tmp}/p.fa", "-n", str(args.queries), "-s", "4",
                        "-N", "10000000"], check=True, capture_output=True)
        print(json.dumps(case(tmp, "protein", f"{tmp}/p.fa", ["-l", "300"], 127, False, args.reps)), flush=True)
        os.remove(f"{tmp}/p.fa")
        subprocess.run([BIN_PATH, "synth", "-q", f"{tmp}/d.fa", "-d", f"{tmp}/db.fa", "-n", str(args.reads),
                        "-N", "100000", "-s", "5", "-t", "dna", "-l", "150"], check=True, capture_output=True)
        print(json.dumps(case(tmp, "dna", f"{tmp}/d.fa", ["-t", "d", "-l", "150"], 50, True, args.reps)), flush=True)


if __name__ == "__main__":
    main()
