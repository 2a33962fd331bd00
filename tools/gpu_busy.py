"""GPU busy fraction per session run from a rocprofv3 kernel trace: the union
of kernel intervals over each run's span (first K1 kernel of the run to the
first of the next, the last run to its last kernel), and the idle gaps above a
threshold with the kernels on either side.

    python tools/gpu_busy.py gpurun_out/x/run_kernel_trace.csv --chunks 1 [--gaps 50]

--chunks: query chunks per run (a run launches k_seed_lists once per chunk);
--skip: runs to leave out at the start (the first run's allocations).
"""
from __future__ import annotations

import argparse
import csv


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--chunks", type=int, default=1)
    ap.add_argument("--skip", type=int, default=1)
    ap.add_argument("--gaps", type=float, default=0.0, help="print idle gaps above this many microseconds")
    args = ap.parse_args()
    ks = []
    with open(args.trace) as f:
        for r in csv.DictReader(f):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ks.sort()
    starts = [k[0] for k in ks if k[2].startswith("ghostm::kern::k_seed_lists")]
    run_starts = starts[:: args.chunks]
    for n, t0 in enumerate(run_starts):
        if n < args.skip:
            continue
        t1 = run_starts[n + 1] if n + 1 < len(run_starts) else max(k[1] for k in ks)
        busy, cur_end, gaps, prev = 0, t0, [], None
        for s, e, name in ks:
            if e <= t0 or s >= t1:
                continue
            s, e = max(s, t0), min(e, t1)
            if s > cur_end:
                if prev is not None and (s - cur_end) / 1e3 > args.gaps > 0:
                    gaps.append(((s - cur_end) / 1e3, prev, name))
            busy += max(0, e - max(s, cur_end))
            cur_end = max(cur_end, e)
            prev = name
        span = t1 - t0
        print(f"run {n}: span {span / 1e6:.3f} ms, kernels busy {busy / 1e6:.3f} ms ({busy / span:.1%})")
        for g, a, b in gaps:
            print(f"    idle {g:8.1f} us  after {a[:60]}  before {b[:60]}")


if __name__ == "__main__":
    main()
