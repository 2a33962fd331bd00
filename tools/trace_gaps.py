"""GPU idle gaps in a rocprofv3 kernel trace (run_kernel_trace.csv): prints every
gap longer than --min-ms between consecutive kernels and the kernel that ends it,
plus the busy fraction over the traced span.

    python tools/trace_gaps.py gpurun_out/prof_r1/trace/run_kernel_trace.csv
"""
from __future__ import annotations

import argparse
import csv


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--min-ms", type=float, default=0.3)
    args = ap.parse_args()
    with open(args.trace, newline="") as f:
        ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:48])
                    for r in csv.DictReader(f))
    if not ev:
        return
    t0 = ev[0][0]
    prev_end = ev[0][1]
    busy = ev[0][1] - ev[0][0]
    idle = 0
    for s, e, name in ev[1:]:
        gap = s - prev_end
        if gap > 0:
            idle += gap
        if gap > args.min_ms * 1e6:
            print(f"at {(prev_end - t0) / 1e6:9.1f} ms  gap {gap / 1e6:7.2f} ms  before {name}")
        busy += max(0, e - max(s, prev_end))
        prev_end = max(prev_end, e)
    span = prev_end - t0
    print(f"span {span / 1e6:.1f} ms, busy {busy / 1e6:.1f} ms ({busy / span:.1%}), idle {idle / 1e6:.1f} ms")


if __name__ == "__main__":
    main()
