"""Pin the FULL-size BASELINE workloads to the reference CPU program (SURVEY.md
§8 c4(4)): sha256, line and byte counts of the reference `aln` output for the
whole synthetic cfg2 (substitute) / cfg3 / cfg4 / cfg5 inputs, written to
tests/golden/full_golden.json. bench.py compares the text of its last timed
step against these (`full_output_matches_reference`), and the scale tests use
the cfg2 entry.

Runs ONLY in the build container, where oracle/_ref/ghostm_ref is compiled from
/root/reference (oracle/Makefile). The reference aligner is single-threaded, so
the query set is cut into P contiguous ranges (`ghostm synth -f first -n count`
writes exactly the records first..first+count-1 of the full set: each query is a
function of (seed, index) only), each range is formatted and searched by its own
reference process, and the outputs are concatenated in range order. Queries are
independent and protein queries form singleton name groups, so this equals the
single-process output (reference aligner.cpp:697-700; SURVEY.md Appendix A.6;
the split is re-checked on every run against a one-process run of the first
range's first queries).

    python tests/golden/make_full_golden.py cfg2 cfg3 [cfg4 cfg5] [-P 6]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import cases  # noqa: E402

from ghostm_amd.workloads import PAM250, TESTSET_DB, WORKLOADS, make_db, make_queries  # noqa: E402

OUT = os.path.join(HERE, "full_golden.json")


def run(*a, **kw):
    return subprocess.run(list(a), check=True, capture_output=True, **kw)


def reference_output(name: str, procs: int, tmp: str) -> dict:
    w = WORKLOADS[name]
    root = os.path.join(tmp, name)
    db = make_db(name, os.path.join(root, "db"), exe=cases.REF)
    n = w["queries"]
    per = (n + procs - 1) // procs
    parts = []
    for k in range(procs):
        cnt = min(per, n - k * per)
        if cnt <= 0:
            break
        parts.append((k * per, cnt, os.path.join(root, f"part{k}")))
    t0 = time.time()
    running = []
    for first, cnt, d in parts:
        q = make_queries(name, d, first, cnt, exe=cases.REF)
        running.append(subprocess.Popen(["nice", "-n", "5", cases.REF, "aln", "-i", q, "-d", db, "-o", f"{d}/out"]
                                        + w["aln"], stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL))
    if any(p.wait() for p in running):
        raise SystemExit(f"{name}: a reference process failed")
    wall = time.time() - t0
    h = hashlib.sha256()
    lines = nbytes = 0
    for _, _, d in parts:
        with open(f"{d}/out", "rb") as f:
            for blk in iter(lambda: f.read(1 << 22), b""):
                h.update(blk)
                lines += blk.count(b"\n")
                nbytes += len(blk)
    # the split is output-invariant: one process over the first 2 x 500 queries
    # equals the first two 500-query ranges concatenated
    chk = os.path.join(root, "check")
    a = [make_queries(name, os.path.join(chk, s), f, 500, exe=cases.REF) for s, f in (("a", 0), ("b", 500))]
    whole = make_queries(name, os.path.join(chk, "ab"), 0, 1000, exe=cases.REF)
    outs = []
    for q in a + [whole]:
        run(cases.REF, "aln", "-i", q, "-d", db, "-o", q + ".out", *w["aln"])
        outs.append(open(q + ".out", "rb").read())
    if outs[0] + outs[1] != outs[2]:
        raise SystemExit(f"{name}: query-range split changed the output")
    return {"sha256": h.hexdigest(), "lines": lines, "bytes": nbytes, "queries": n,
            "query_synth": ["-n", str(n)] + [os.path.basename(x) if x in (TESTSET_DB, PAM250) else x
                                              for x in w["synth"]],
            "db": [os.path.basename(x) if isinstance(x, str) and os.path.isabs(x) else x for x in w["db"]],
            "qry": w["qry"],
            "aln": [os.path.basename(x) if x == PAM250 else x for x in w["aln"]],
            "reference_processes": len(parts), "reference_wall_s": round(wall, 1)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("names", nargs="+", choices=sorted(WORKLOADS))
    ap.add_argument("-P", type=int, default=6)
    args = ap.parse_args()
    if not os.path.exists(cases.REF):
        raise SystemExit("oracle/_ref/ghostm_ref missing: make -C oracle ref")
    data = {}
    if os.path.exists(OUT):
        with open(OUT) as f:
            data = json.load(f)
    data.setdefault("generator", "tests/golden/make_full_golden.py")
    data.setdefault("reference", "oracle/_ref/ghostm_ref (reference CPU path, g++ -O2), P query-range processes")
    tmp = tempfile.mkdtemp(prefix="ghostm_full_golden_", dir=os.environ.get("GHOSTM_GOLDEN_TMP"))
    for name in args.names:
        t = time.time()
        data[name] = reference_output(name, args.P, tmp)
        print(f"{name}: {data[name]['lines']} lines, {time.time() - t:.0f} s", flush=True)
        with open(OUT, "w") as f:
            json.dump(data, f, indent=1, sort_keys=True)
    subprocess.run(["rm", "-rf", tmp])


if __name__ == "__main__":
    main()
