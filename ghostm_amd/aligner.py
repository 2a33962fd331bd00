"""Python face of the native `aln` engine, mirroring the reference C++ API.

    Aligner().execute(["aln", "-i", q, "-d", db, "-o", out, ...])
        reference Aligner::Execute (aligner.cpp:65-223) — same flags, same output.

    Session(argv)            inputs loaded once and resident in HBM; .run() is the
                             hot path (seed -> score -> merge -> traceback ->
                             E-value text), repeatable, with .output(), .hits(),
                             .stats().

Everything runs in libghostm_hip.so (HIP kernels for gfx950 + host merge); this
module only marshals arguments.
"""
from __future__ import annotations

import ctypes
import subprocess
from typing import Sequence

import numpy as np

from . import native

HIT_DTYPE = np.dtype(
    [
        ("query_id", "<u4"),
        ("db_id", "<u4"),
        ("score", "<u4"),
        ("db_start", "<u4"),
        ("db_end", "<u4"),
        ("aln_len", "<u4"),
        ("aln_match", "<u4"),
        ("seq_id", "<f4"),
    ]
)


class GhostmError(RuntimeError):
    pass


class Aligner:
    """reference class Aligner (aligner.h:63-92): Execute(argc, argv)."""

    def execute(self, argv: Sequence[str]) -> int:
        lib = native.load()
        args = list(argv)
        return int(lib.GhostmAlignMain(len(args), native.argv_array(args)))


class Session:
    """`shard=(rank, world)`: search only that shard of the query set (one process
    per GPU, GhostmSessionCreateShard); rank-order concatenation of the shards'
    outputs is the unsharded output.

    `exchange`: an all-gather `f(send: bytes, sizes: list[int]) -> bytes` over
    the ranks (ghostm_amd.shard.torch_allgather): the shard then reads and
    counts only its own queries, and the ranks agree on the unsharded batch
    plan through it (GhostmSessionCreateShardEx). Without it, the shard counts
    every query of the set itself."""

    def __init__(self, argv: Sequence[str], shard: tuple[int, int] | None = None, exchange=None):
        lib = native.load()
        args = ["aln"] + list(argv)
        self._argv = native.argv_array(args)
        if shard is None:
            self._h = lib.GhostmSessionCreate(len(args), self._argv)
        elif exchange is None:
            self._h = lib.GhostmSessionCreateShard(len(args), self._argv, int(shard[0]), int(shard[1]))
        else:
            world = int(shard[1])
            errors = []

            def gather(_ctx, send, nbytes, recv, recv_bytes):
                try:
                    sizes = [int(recv_bytes[r]) for r in range(world)]
                    data = ctypes.string_at(send, nbytes) if nbytes else b""
                    out = exchange(data, sizes)
                    if len(out) != sum(sizes):
                        raise GhostmError(f"all-gather returned {len(out)} bytes, expected {sum(sizes)}")
                    if out:
                        ctypes.memmove(recv, out, len(out))
                    return 0
                except BaseException as e:  # noqa: BLE001 (reported through the C ABI)
                    errors.append(e)
                    return 1

            fn = native.ALLGATHER_FN(gather)  # alive for the duration of the call
            self._h = lib.GhostmSessionCreateShardEx(len(args), self._argv, int(shard[0]), world,
                                                     ctypes.cast(fn, ctypes.c_void_p), None)
            if errors:
                raise errors[0]
        if not self._h:
            raise GhostmError(native.last_error())

    def shard_range(self) -> tuple[int, int]:
        b, e = ctypes.c_uint64(), ctypes.c_uint64()
        native.load().GhostmSessionShardRange(self._h, ctypes.byref(b), ctypes.byref(e))
        return b.value, e.value

    def hit_capacity(self) -> int:
        """The most hit records one run can return (name groups x max(-b, 1),
        GhostmSessionHitCapacity): the size of a fixed gather buffer."""
        return int(native.load().GhostmSessionHitCapacity(self._h))

    def run(self, to_file: bool = False) -> None:
        """The search; to_file also writes the -o file while it runs
        (GhostmSessionRunToFile), after which write() is a no-op."""
        lib = native.load()
        rc = lib.GhostmSessionRunToFile(self._h) if to_file else lib.GhostmSessionRun(self._h)
        if rc != 0:
            raise GhostmError(native.last_error())

    def output(self) -> bytes:
        lib = native.load()
        n = lib.GhostmSessionOutput(self._h, None, 0)
        buf = ctypes.create_string_buffer(n)
        lib.GhostmSessionOutput(self._h, buf, n)
        return buf.raw[:n]

    def write(self) -> None:
        if native.load().GhostmSessionWrite(self._h) != 0:
            raise GhostmError(native.last_error())

    def hits(self) -> np.ndarray:
        lib = native.load()
        n = lib.GhostmSessionHits(self._h, None, 0)
        out = np.zeros(n, dtype=HIT_DTYPE)
        if n:
            lib.GhostmSessionHits(self._h, out.ctypes.data_as(ctypes.POINTER(native.GhostmHit)), n)
        return out

    def device_hits(self, device="cuda"):
        """The hit records as a torch uint8 tensor on this session's GPU (32 bytes
        per record, HIT_DTYPE layout), copied device-to-device — the payload of
        the multi-GPU gather."""
        import torch

        lib = native.load()
        n = lib.GhostmSessionDeviceHits(self._h, None, 0)
        if n == ctypes.c_size_t(-1).value:
            raise GhostmError(native.last_error())
        out = torch.empty(max(n, 1) * HIT_DTYPE.itemsize, dtype=torch.uint8, device=device)
        if n:
            torch.cuda.synchronize(out.device)
            if lib.GhostmSessionDeviceHits(self._h, ctypes.c_void_p(out.data_ptr()), n) != n:
                raise GhostmError(native.last_error())
        return out[: n * HIT_DTYPE.itemsize]

    def device_hits_into(self, dst, cap: int) -> int:
        """Copies the hit records of the last run device-to-device into `dst` (a
        uint8 torch tensor on this session's GPU with room for `cap` records);
        returns their number. Raises if there are more than `cap`."""
        import torch

        lib = native.load()
        n = lib.GhostmSessionDeviceHits(self._h, None, 0)
        if n == ctypes.c_size_t(-1).value:
            raise GhostmError(native.last_error())
        if n > cap or dst.numel() < n * HIT_DTYPE.itemsize:
            raise GhostmError(f"{n} hit records do not fit the destination ({cap} records)")
        if n:
            torch.cuda.synchronize(dst.device)
            if lib.GhostmSessionDeviceHits(self._h, ctypes.c_void_p(dst.data_ptr()), n) != n:
                raise GhostmError(native.last_error())
        return n

    def stats(self) -> dict:
        st = native.GhostmStats()
        # the sized call: a library built with more fields writes only ours
        native.load().GhostmSessionStatsSized(self._h, ctypes.byref(st), ctypes.sizeof(st))
        return st.as_dict()

    def close(self) -> None:
        if self._h:
            native.load().GhostmSessionDestroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def run_cli(args: Sequence[str], **kw) -> subprocess.CompletedProcess:
    """Run the native `ghostm` binary (db | qry | aln | synth)."""
    return subprocess.run([native.BIN_PATH] + list(args), check=True, capture_output=True, **kw)


def format_db(fasta: str, prefix: str, *extra: str) -> None:
    run_cli(["db", "-i", fasta, "-o", prefix, *extra])


def format_queries(fasta: str, prefix: str, *extra: str) -> None:
    run_cli(["qry", "-i", fasta, "-o", prefix, *extra])


def synth(db_fasta: str | None, query_fasta: str | None, nq: int, db_residues: int, seed: int,
          *extra: str) -> None:
    args = ["synth", "-n", str(nq), "-N", str(db_residues), "-s", str(seed)]
    if db_fasta:
        args += ["-d", db_fasta]
    if query_fasta:
        args += ["-q", query_fasta]
    run_cli(args + list(extra))
