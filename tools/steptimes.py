"""Per-step wall times of the bench workload (cfg4 by default) through one
Session: the distribution behind bench.py's mean, for spotting intermittent
stalls. Usage: python tools/steptimes.py [--steps N] [--workdir DIR]"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from ghostm_amd.aligner import Session  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=8)
ap.add_argument("--workdir", default="/tmp/ghostm_steptimes")
args = ap.parse_args()
if not os.path.exists(os.path.join(args.workdir, "q.inf")):
    bench.make_data(args.workdir, 1000000, 10000000, 0, seed=4)
w = args.workdir
s = Session(["-i", f"{w}/q", "-d", f"{w}/db", "-o", f"{w}/out", "-D", "0"])
for k in range(args.steps):
    t = time.perf_counter()
    s.run()
    dt = time.perf_counter() - t
    st = s.stats()
    print(f"step {k} {dt * 1e3:8.1f} ms  seed {st['seconds_seed'] * 1e3:6.1f} score {st['seconds_score'] * 1e3:6.1f} "
          f"tb {st['seconds_traceback'] * 1e3:6.1f} merge {st['seconds_merge'] * 1e3:6.1f} "
          f"out {st['seconds_output'] * 1e3:6.1f}", flush=True)
