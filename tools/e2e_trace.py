"""Host timeline of end-to-end `aln` runs as bench.py's end_to_end leg makes
them (dirty pages written back, a settle pause, then session create, the search
with the output file streamed, the file complete), with GHOSTM_TRACE=1: the
library prints each run's marks (create's reads and uploads, K1..K3, every
segment's formatting and the writer's w_begin/w_end) to stderr.

    GHOSTM_TRACE=1 python tools/e2e_trace.py --preset cfg2 --runs 5 --workdir /tmp/d 2> trace.log
"""
from __future__ import annotations

import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from ghostm_amd import workloads  # noqa: E402
from ghostm_amd.aligner import Session  # noqa: E402


def cpu_stat() -> dict:
    """The cgroup's CPU counters (cgroup v2 cpu.stat): throttling shows as
    nr_throttled / throttled_usec growing across a run."""
    out = {}
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            for line in f:
                k, v = line.split()
                out[k] = int(v)
    except OSError:
        pass
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="cfg2")
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--workdir", default="/tmp/ghostm_e2e_trace")
    ap.add_argument("--settle", type=float, default=1.0)
    args = ap.parse_args()
    w = workloads.WORKLOADS[args.preset]
    db = workloads.make_db(args.preset, os.path.join(args.workdir, "db"))
    q = workloads.make_queries(args.preset, os.path.join(args.workdir, "q"), 0, w["queries"])
    out = os.path.join(args.workdir, "out")
    argv = ["-i", q, "-d", db, "-o", out, "-D", "0"] + list(w["aln"])
    with Session(argv) as s:  # warm: the HIP runtime, the device pool
        s.run()
    for k in range(args.runs):
        if os.path.exists(out):
            os.remove(out)
        os.sync()
        time.sleep(args.settle)
        print(f"=== run {k}", file=sys.stderr, flush=True)
        c0 = cpu_stat()
        t0 = time.perf_counter()
        with Session(argv) as s:
            t1 = time.perf_counter()
            s.run(to_file=True)
            t2 = time.perf_counter()
        c1 = cpu_stat()
        d = {k: c1[k] - c0.get(k, 0) for k in ("nr_throttled", "throttled_usec", "usage_usec") if k in c1}
        print(f"e2e run {k}: create {1e3 * (t1 - t0):.2f} ms, run+write {1e3 * (t2 - t1):.2f} ms, "
              f"total {1e3 * (t2 - t0):.2f} ms, file {os.path.getsize(out)} bytes, cpu {d}", flush=True)


if __name__ == "__main__":
    main()
