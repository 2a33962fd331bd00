"""Query sharding and the single hit-record gather of the multi-GPU path
(SURVEY.md §8 e1).

One process per GPU: rank r searches its own contiguous query range against a
full DB replica; nothing crosses ranks on the data path. At the end the 32-byte
hit records (`GhostmHit`, include/ghostm_hip.h) of every rank are gathered to
rank 0 in rank order — with contiguous shards that is the single-GPU output
order. Over RCCL (backend "nccl") on GPUs; the same code runs over gloo on CPU
for the tests.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np


def balanced_cuts(weights: Sequence[int], names: Sequence[str], world: int) -> list[int]:
    """Cut points c[0]=0 <= ... <= c[world]=n splitting queries into `world`
    contiguous shards of about equal total weight (e.g. residues), never inside a
    group of consecutive equal names — the reference merges such a group (DNA
    frames) into one result list (aligner.cpp:697-700), so it must stay on one rank."""
    n = len(weights)
    if len(names) != n:
        raise ValueError("weights and names differ in length")
    if world < 1:
        raise ValueError("world must be >= 1")
    # group starts: a query starts a group unless its name equals the previous one
    starts = [i for i in range(n) if i == 0 or names[i] != names[i - 1]]
    prefix = [0]
    for w in weights:
        prefix.append(prefix[-1] + int(w))
    total = prefix[-1]
    cuts = [0]
    for r in range(1, world):
        # first group start at or after the previous cut whose prefix weight
        # reaches total * r / world (integer comparison, as GhostmShardCuts)
        best = n
        for s in starts:
            if s >= cuts[-1] and prefix[s] * world >= total * r:
                best = s
                break
        cuts.append(max(cuts[-1], best))
    cuts.append(n)
    return cuts


def gather_device_records(payload, dist, itemsize: int):
    """One gather of every rank's hit records, already on its GPU as a uint8
    tensor (Session.device_hits), to rank 0 over RCCL — no host copies on any
    rank. Returns rank 0's list of per-rank uint8 tensors (device), None elsewhere."""
    import torch

    world = dist.get_world_size()
    rank = dist.get_rank()
    n = torch.tensor([payload.numel()], device=payload.device, dtype=torch.int64)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    cap = max(int(s.item()) for s in sizes)
    buf = payload
    if payload.numel() != cap or cap == 0:
        buf = torch.zeros(max(cap, itemsize), dtype=torch.uint8, device=payload.device)
        buf[: payload.numel()] = payload
    gathered = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, gathered, dst=0)
    if rank != 0:
        return None
    return [g[: int(s.item())] for g, s in zip(gathered, sizes)]


class RecordGather:
    """The single data-path collective of a step: every rank
    sends a fixed-capacity buffer of `cap` 32-byte hit records plus one header
    record (its count), and rank 0 receives all of them in one gather — no size
    exchange first, since cap (shard queries x -b, the most a shard can return)
    is fixed for the session. The buffers are allocated once."""

    def __init__(self, dist, cap_records: int, itemsize: int, device):
        import torch

        self.dist = dist
        self.itemsize = itemsize
        self.cap = int(cap_records)
        self.world = dist.get_world_size()
        self.rank = dist.get_rank()
        self.buf = torch.zeros((self.cap + 1) * itemsize, dtype=torch.uint8, device=device)
        self.parts = [torch.empty_like(self.buf) for _ in range(self.world)] if self.rank == 0 else None

    def payload(self):
        """The record area (cap records), to be filled in place."""
        return self.buf[self.itemsize:]

    def set_count(self, n: int) -> None:
        import torch

        if n > self.cap:
            raise ValueError(f"{n} hit records exceed the gather capacity {self.cap}")
        self.buf[:8].copy_(torch.tensor([n], dtype=torch.int64).view(torch.uint8))

    def gather(self) -> None:
        self.dist.gather(self.buf, self.parts, dst=0)

    def records(self):
        """Rank 0: every rank's records (uint8 tensors, device) in rank order."""
        import torch

        if self.parts is None:
            return None
        out = []
        for p in self.parts:
            n = int(p[:8].cpu().view(torch.int64)[0])
            if n > self.cap:
                raise ValueError("gathered header exceeds the capacity")
            out.append(p[self.itemsize: self.itemsize + n * self.itemsize])
        return out


def gather_hits(hits: np.ndarray, dist, device) -> list[np.ndarray] | None:
    """Gather every rank's hit records (a structured array of any dtype) to rank 0.
    Returns the per-rank arrays in rank order on rank 0, None elsewhere. Sizes
    differ per rank, so an all_gather of the byte counts precedes one gather of
    buffers padded to the largest."""
    import torch

    world = dist.get_world_size()
    rank = dist.get_rank()
    raw = np.ascontiguousarray(hits).view(np.uint8).reshape(-1)
    payload = torch.from_numpy(raw.copy()).to(device)
    n = torch.tensor([payload.numel()], device=device, dtype=torch.int64)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    cap = max(int(s.item()) for s in sizes)
    buf = torch.zeros(max(cap, 1), dtype=torch.uint8, device=device)
    buf[: payload.numel()] = payload
    gathered = [torch.zeros_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, gathered, dst=0)
    if rank != 0:
        return None
    return [g[: int(s.item())].cpu().numpy().view(hits.dtype) for g, s in zip(gathered, sizes)]


def gather_bytes(data: bytes, dist, device="cpu") -> list[bytes] | None:
    """Gather every rank's byte string (e.g. its formatted output) to rank 0 in
    rank order; None on other ranks."""
    import torch

    payload = torch.frombuffer(bytearray(data), dtype=torch.uint8) if data else torch.zeros(0, dtype=torch.uint8)
    parts = gather_device_records(payload.to(device), dist, 1)
    if parts is None:
        return None
    return [p.cpu().numpy().tobytes() for p in parts]


def torch_allgather(dist, device="cpu", group=None):
    """The all-gather a rank-local shard session needs (Session(exchange=...),
    GhostmSessionCreateShardEx) over torch.distributed: every rank's byte buffer
    (sizes[r] bytes from rank r, known to all ranks) concatenated in rank order.
    Buffers are padded to the largest for one all_gather."""
    import torch

    def allgather(send: bytes, sizes: list[int]) -> bytes:
        world = dist.get_world_size(group)
        if len(sizes) != world:
            raise ValueError("one size per rank")
        cap = max(max(sizes), 1)
        buf = torch.zeros(cap, dtype=torch.uint8)
        if send:
            buf[: len(send)] = torch.frombuffer(bytearray(send), dtype=torch.uint8)
        buf = buf.to(device)
        parts = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(parts, buf, group=group)
        return b"".join(p[:n].cpu().numpy().tobytes() for p, n in zip(parts, sizes))

    return allgather


def shard_cuts_native(weights, group_start, world: int) -> list[int]:
    """GhostmShardCuts (the C ABI the shard sessions use), for tests."""
    import ctypes

    from . import native

    w = np.ascontiguousarray(weights, dtype=np.uint32)
    g = np.ascontiguousarray(group_start, dtype=np.uint8)
    cuts = np.zeros(world + 1, dtype=np.uint64)
    rc = native.load().GhostmShardCuts(len(w), w.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                       g.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), world,
                                       cuts.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    if rc != 0:
        raise ValueError(native.last_error())
    return [int(x) for x in cuts]
