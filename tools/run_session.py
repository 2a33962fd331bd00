"""Run a preset's session a few times without checks (kernel-timing variants:
rocprofv3 around it, GHOSTM_LIB_PATH selecting the library build).

    python tools/run_session.py --preset cfg4 --runs 2 --workdir /tmp/data
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


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="cfg4")
    ap.add_argument("--runs", type=int, default=2)
    ap.add_argument("--workdir", default="/tmp/ghostm_run_session")
    args = ap.parse_args()
    w = workloads.WORKLOADS[args.preset]
    db = workloads.make_db(args.preset, os.path.join(args.workdir, "db"))
    q = workloads.make_queries(args.preset, os.path.join(args.workdir, "q"), 0, w["queries"])
    with Session(["-i", q, "-d", db, "-o", os.devnull, "-D", "0"] + list(w["aln"])) as s:
        for _ in range(args.runs):
            t = time.perf_counter()
            s.run()
            print(f"run {1e3 * (time.perf_counter() - t):.1f} ms, hits {s.stats()['hits']}", flush=True)


if __name__ == "__main__":
    main()
