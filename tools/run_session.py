"""Run a preset's session a few times without checks (kernel-timing variants:
rocprofv3 around it, GHOSTM_LIB_PATH selecting the library build). --kfd
prints this process's KFD counters (/sys/class/kfd/kfd/proc/<pid>/: queue
eviction time, memory use) after the create and after each run, to tell a
queue eviction from other waits.

    python tools/run_session.py --preset cfg4 --runs 2 --workdir /tmp/data
"""
from __future__ import annotations

import argparse
import glob
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from ghostm_amd import workloads  # noqa: E402
from ghostm_amd.aligner import Session  # noqa: E402


def kfd_counters() -> dict:
    base = f"/sys/class/kfd/kfd/proc/{os.getpid()}"
    out = {}
    for f in sorted(glob.glob(base + "/**", recursive=True)):
        if os.path.isfile(f):
            try:
                with open(f) as fh:
                    out[os.path.relpath(f, base)] = fh.read().strip()
            except OSError as e:
                out[os.path.relpath(f, base)] = f"<{e.strerror}>"
    return out if out else {"kfd": f"no {base}"}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="cfg4")
    ap.add_argument("--runs", type=int, default=2)
    ap.add_argument("--workdir", default="/tmp/ghostm_run_session")
    ap.add_argument("--kfd", action="store_true")
    ap.add_argument("--out", default=os.devnull, help="output file (-o); bench.py writes a real file")
    ap.add_argument("--queries", type=int, default=0, help="the first N queries of the preset (0: all)")
    args = ap.parse_args()
    w = workloads.WORKLOADS[args.preset]
    db = workloads.make_db(args.preset, os.path.join(args.workdir, "db"))
    q = workloads.make_queries(args.preset, os.path.join(args.workdir, "q"), 0, args.queries or w["queries"])
    with Session(["-i", q, "-d", db, "-o", args.out, "-D", "0"] + list(w["aln"])) as s:
        if args.kfd:
            print("kfd after create", kfd_counters(), flush=True)
        for _ in range(args.runs):
            t = time.perf_counter()
            s.run()
            print(f"run {1e3 * (time.perf_counter() - t):.1f} ms, hits {s.stats()['hits']}", flush=True)
            if args.kfd:
                print("kfd", kfd_counters(), flush=True)


if __name__ == "__main__":
    main()
