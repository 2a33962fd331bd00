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


def single_process_output(name: str, tmp: str) -> dict:
    """One reference process over the whole query set (the multi-batch pins:
    batch cuts depend on the whole chunk), with -v, whose per-batch log lines
    give the number of batches the reference ran."""
    w = WORKLOADS[name]
    root = os.path.join(tmp, name)
    db = make_db(name, os.path.join(root, "db"), exe=cases.REF)
    n = w["queries"]
    q = make_queries(name, os.path.join(root, "q"), 0, n, exe=cases.REF)
    t0 = time.time()
    log = run("nice", "-n", "5", cases.REF, "aln", "-i", q, "-d", db, "-o", f"{root}/out", "-v", *w["aln"]).stdout
    wall = time.time() - t0
    batches = log.count(b"|Calculate scores")
    h = hashlib.sha256()
    with open(f"{root}/out", "rb") as f:
        data = f.read()
    h.update(data)
    return {"sha256": h.hexdigest(), "lines": data.count(b"\n"), "bytes": len(data), "queries": n,
            "query_synth": ["-n", str(n)] + [os.path.basename(x) if x in (TESTSET_DB, PAM250) else x
                                              for x in w["synth"]],
            "db": [os.path.basename(x) if isinstance(x, str) and os.path.isabs(x) else x for x in w["db"]],
            "qry": w["qry"],
            "aln": [os.path.basename(x) if x == PAM250 else x for x in w["aln"]],
            "reference_batches": batches,
            "reference_processes": 1, "reference_wall_s": round(wall, 1)}


def restatement_check(name: str, pin: dict, tmp: str) -> bool:
    """The builder's CPU restatement (oracle/_build/ghostm_oracle) on the same
    single-process workload, against the reference pin."""
    w = WORKLOADS[name]
    root = os.path.join(tmp, name + "_restated")
    db = make_db(name, os.path.join(root, "db"))
    q = make_queries(name, os.path.join(root, "q"), 0, w["queries"])
    run("nice", "-n", "5", cases.ORACLE, "aln", "-i", q, "-d", db, "-o", f"{root}/out", *w["aln"])
    h = hashlib.sha256()
    with open(f"{root}/out", "rb") as f:
        h.update(f.read())
    return h.hexdigest() == pin["sha256"]


def reference_output(name: str, procs: int, tmp: str) -> dict:
    w = WORKLOADS[name]
    if w.get("single_process"):
        return single_process_output(name, tmp)
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
    ap.add_argument("--check-restatement", action="store_true",
                    help="only run the restatement on already pinned single-process workloads")
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
    if args.check_restatement:
        from concurrent.futures import ThreadPoolExecutor

        names = [n for n in args.names if n in data]
        with ThreadPoolExecutor(max(1, min(len(names), args.P))) as pool:
            oks = list(pool.map(lambda n: restatement_check(n, data[n], tmp), names))
        for n, ok in zip(names, oks):
            print(f"{n}: restatement {'equals' if ok else 'DIFFERS FROM'} the reference pin", flush=True)
            data[n]["restatement_matches"] = ok
        with open(OUT, "w") as f:
            json.dump(data, f, indent=1, sort_keys=True)
        subprocess.run(["rm", "-rf", tmp])
        return
    # single-process pins run side by side (one reference process each); the
    # split pins one after another (each uses P processes)
    single = [n for n in args.names if WORKLOADS[n].get("single_process")]
    split = [n for n in args.names if n not in single]

    def one(name):
        t = time.time()
        res = reference_output(name, args.P, tmp)
        print(f"{name}: {res['lines']} lines, {time.time() - t:.0f} s", flush=True)
        return name, res

    from concurrent.futures import ThreadPoolExecutor

    with ThreadPoolExecutor(max(1, min(len(single), args.P))) as pool:
        results = list(pool.map(one, single))
    results += [one(n) for n in split]
    for name, res in results:
        data[name] = res
    with open(OUT, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)
    subprocess.run(["rm", "-rf", tmp])


if __name__ == "__main__":
    main()
