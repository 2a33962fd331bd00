"""One process per GPU for `bench.py --gpus N`, without an
external torchrun, plus the per-rank host placement and failure agreement the
multi-GPU path needs.

* `spawn`: the parent starts N children of the same script before anything
  touches the GPU (it imports no torch and never execs), each with RANK,
  LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR = 127.0.0.1 and a free
  MASTER_PORT. The children inherit stdout, so rank 0's JSON line is the
  parent's output. The parent waits; when a child fails it gives the others a
  grace period (they fail on their own through `agree`) and then kills them.
  Its exit status is the first failing child's, else 0.
* `bind_numa`: pins every thread of a rank to the CPUs next to its GPU
  (`/sys/bus/pci/devices/<bdf>/local_cpulist`), split disjointly among the
  ranks of this host that share those CPUs, and sets GHOSTM_THREADS to the
  rank's share so the library's formatting pool matches it.
* `agree`: every rank contributes an ok flag to one MIN all-reduce, so one
  rank's exception stops every rank instead of leaving its peers in the next
  collective.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time

LAUNCH_ENV = "GHOSTM_LAUNCHED_BY_BENCH"


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def world_from_env(gpus: int | None) -> tuple[int, bool]:
    """(world size, spawn?) for `--gpus`: WORLD_SIZE set (torchrun or our own
    children) must equal --gpus when both are given; WORLD_SIZE unset with
    --gpus N > 1 means this process launches the N ranks itself."""
    env = os.environ.get("WORLD_SIZE")
    if env is not None:
        world = int(env)
        if gpus is not None and gpus != world:
            raise SystemExit(f"bench: --gpus {gpus} but WORLD_SIZE={world}; they must agree")
        return world, False
    n = 1 if gpus is None else gpus
    if n < 1:
        raise SystemExit("bench: --gpus must be >= 1")
    return n, n > 1


def spawn(argv: list[str], n: int, grace_s: float = 60.0, extra_env: dict | None = None) -> int:
    """Run `python argv...` as n ranks on this host; returns the exit status."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update(extra_env or {})
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                    "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), LAUNCH_ENV: "1"})
        # only rank 0 reports on stdout; the other ranks' output goes to stderr
        procs.append(subprocess.Popen([sys.executable] + argv, env=env, stdout=None if r == 0 else sys.stderr))
    status = 0
    failed_at = None
    try:
        while True:
            alive = [p for p in procs if p.poll() is None]
            for p in procs:
                if p.returncode not in (None, 0) and status == 0:
                    status = p.returncode if p.returncode > 0 else 128 - p.returncode
                    failed_at = time.monotonic()
                    print(f"[launch] rank {procs.index(p)} exited with {p.returncode}", file=sys.stderr, flush=True)
            if not alive:
                break
            if failed_at is not None and time.monotonic() - failed_at > grace_s:
                for p in alive:
                    print(f"[launch] killing rank {procs.index(p)} after a peer failed", file=sys.stderr, flush=True)
                    p.send_signal(signal.SIGTERM)
                deadline = time.monotonic() + 10
                for p in alive:
                    try:
                        p.wait(timeout=max(0.1, deadline - time.monotonic()))
                    except subprocess.TimeoutExpired:
                        p.kill()
                        p.wait()
                break
            time.sleep(0.2)
    except KeyboardInterrupt:
        for p in procs:
            if p.poll() is None:
                p.kill()
        raise
    return status


def parse_cpulist(text: str) -> list[int]:
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]."""
    cpus: list[int] = []
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            cpus.extend(range(int(a), int(b) + 1))
        else:
            cpus.append(int(part))
    return cpus


def cgroup_cpus() -> int | None:
    """The cgroup v2 CPU quota in whole CPUs (None = unlimited)."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota == "max":
            return None
        return max(1, -(-int(quota) // int(period)))
    except (OSError, ValueError):
        return None


def gpu_local_cpus(device: int) -> tuple[str | None, list[int] | None]:
    """(PCI address, CPUs local to it) of a GPU of this process, or (None, None)."""
    import torch

    p = torch.cuda.get_device_properties(device)
    bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    try:
        with open(f"/sys/bus/pci/devices/{bdf}/local_cpulist") as f:
            return bdf, parse_cpulist(f.read())
    except OSError:
        return bdf, None


def split_share(cpus: list[int], peers: int, index: int) -> list[int]:
    """The index-th of `peers` disjoint contiguous slices of cpus (each non-empty
    while there are at least as many CPUs as peers; else CPUs are shared)."""
    if not cpus:
        return []
    if peers <= len(cpus):
        per, extra = divmod(len(cpus), peers)
        lo = index * per + min(index, extra)
        return cpus[lo: lo + per + (1 if index < extra else 0)]
    return [cpus[index % len(cpus)]]


def bind_numa(dist, rank: int, device: int) -> dict:
    """Pin this rank to its GPU's local CPUs (disjoint among the ranks of this
    host that share them); returns what was done, for the bench line."""
    allowed = sorted(os.sched_getaffinity(0))
    info: dict = {"rank": rank, "host": os.uname().nodename, "device": device}
    try:
        bdf, local = gpu_local_cpus(device)
    except Exception as e:  # noqa: BLE001 (placement is best effort; reported)
        bdf, local = None, None
        info["error"] = str(e)
    info["pci"] = bdf
    pool = [c for c in (local or allowed) if c in set(allowed)] or allowed
    key = (info["host"], tuple(pool))
    keys = [None] * dist.get_world_size()
    dist.all_gather_object(keys, key)
    sharing = [r for r, k in enumerate(keys) if k == key]
    mine = split_share(pool, len(sharing), sharing.index(rank))
    local_world = sum(1 for k in keys if k[0] == info["host"])
    quota = cgroup_cpus()
    threads = max(1, min(16, len(mine), (quota // local_world) if quota else len(mine)))
    # every thread of the process: sched_setaffinity(0) pins only the calling
    # thread, and the HIP runtime, RCCL and gloo have started theirs by now
    bound, failed = bind_threads(mine)
    info["bound"] = bound > 0 and not failed
    info["threads_bound"] = bound
    if failed:
        info["error"] = f"{len(failed)} thread(s) could not be bound: {failed[0]}"
    os.environ["GHOSTM_THREADS"] = str(threads)
    info.update({"numa_local": local is not None, "cpus": _fmt_cpulist(mine), "threads": threads,
                 "ranks_sharing_cpus": len(sharing)})
    return info


def bind_threads(cpus: list[int]) -> tuple[int, list[str]]:
    """Set the CPU affinity of every thread of this process (each TID under
    /proc/self/task; threads created later inherit it from their creator).
    Returns (threads bound, errors)."""
    try:
        tids = sorted(int(t) for t in os.listdir("/proc/self/task"))
    except OSError:
        tids = [0]
    bound, failed = 0, []
    for tid in tids:
        try:
            os.sched_setaffinity(tid, cpus)
            bound += 1
        except ProcessLookupError:  # the thread ended meanwhile
            continue
        except OSError as e:
            failed.append(f"tid {tid}: {e}")
    return bound, failed


def _fmt_cpulist(cpus: list[int]) -> str:
    out, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(out)


class PeerFailed(RuntimeError):
    pass


def agree(dist, ok: bool, device="cpu", what: str = "step") -> None:
    """One MIN all-reduce of every rank's ok flag; raises PeerFailed on every
    rank if any rank failed (the failing rank raises its own error after)."""
    import torch

    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if int(flag.item()) != 1 and ok:
        raise PeerFailed(f"another rank failed in {what}")
