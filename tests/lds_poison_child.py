"""Child process of tests/test_gpu_lds_poison.py (one process per LDS pattern;
not a test module itself).

Runs with GHOSTM_LIB_PATH = the LDS poison build (libghostm_hip_poison.so: every
kernel fills its whole LDS allocation with GHOSTM_LDS_POISON_PATTERN before its
own code) and checks the golden variants under the kernel forms that read LDS:

  golden:  every golden variant with the default kernels, with the unit-pair
           K2 forced as paired and as consecutive tasks, and with the sparse
           segments' pair-table and 16-row profile K2s forced;
  kernels: every K3 scan mode, every K4 mode, every K1 size class and the
           offset pass (class caps at the dataset's quartiles, slot cap 2), the
           bin table's probe bound lowered to 0 and 1 windows (the table-free
           redo), and the many-segment device pipeline.

Prints one JSON line {"runs": n, "failures": [...]} and exits 1 on a mismatch."""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

import cases  # noqa: E402
from ghostm_amd import native  # noqa: E402
from ghostm_amd.aligner import Session  # noqa: E402


def run(d, opts, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        with Session(["-i", os.path.join(d, "q"), "-d", os.path.join(d, "db"), "-o", os.path.join(d, "x"),
                      "-D", "0"] + list(opts)) as s:
            s.run()
            return s.output(), s.stats()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def caps(d):
    n = cases.k1_list_entries(d)
    return ",".join(str(int(np.percentile(n[n > 0], p))) for p in (25, 50, 75))


def plan(group):
    if group == "golden":
        for ds, var, opts, env in cases.VARIANTS:
            yield ds, var, opts, dict(env), "default"
            for tasks in ("paired", "consecutive"):
                yield ds, var, opts, dict(env, GHOSTM_K2="unit", GHOSTM_K2_TASKS=tasks), f"unit_{tasks}"
            yield ds, var, opts, dict(env, GHOSTM_K2="pair"), "pair"
            yield ds, var, opts, dict(env, GHOSTM_K2="sparse"), "sparse_rows"
        return
    scan_sets = [("syn_small", "default", []), ("syn_dna", "default", []), ("syn_chunks", "default", []),
                 ("protein_testset", "y2", ["-y", "2"]),
                 ("syn_small", "r64_pam250", ["-r", "64", "-M", cases.PAM250, "-y", "2"])]
    for mode in ("default", "priv", "f16frame", "f16plain", "int16", "0"):
        for ds, var, opts in scan_sets:
            yield ds, var, opts, ({} if mode == "default" else {"GHOSTM_K3_SCAN": mode}), f"k3_scan_{mode}"
    for ds, var, opts in scan_sets[:2]:
        yield ds, var, opts, {"GHOSTM_K3_STRIPS": "0"}, "k3_nostrips"
        yield ds, var, opts, {"GHOSTM_K3": "int32"}, "k3_int32"
    for mode in ("thread", "wave", "wave_cap40"):
        env = {"GHOSTM_K4": "thread"} if mode == "thread" else {"GHOSTM_K4": "wave"}
        if mode == "wave_cap40":
            env["GHOSTM_K4_CAP"] = "40"
        for ds, var, opts in [("syn_small", "b20_t1", ["-b", "20", "-t", "1", "-y", "2"]),
                              ("syn_dna", "b5_y2", ["-b", "5", "-y", "2"])]:
            yield ds, var, opts, env, f"k4_{mode}"
    for k1 in ("hash", "merge"):
        for ds, var, opts in [("syn_small", "default", []), ("syn_dna", "default", []),
                              ("syn_short", "default", [])]:
            env = {"GHOSTM_K1_CAPS": "@caps", "GHOSTM_K1_SLOT_CAP": "2"}
            if k1 == "merge":
                env["GHOSTM_K1"] = "merge"
            yield ds, var, opts, env, f"k1_classes_{k1}"
    for ds, var, opts in [("syn_repeat", "default", []), ("syn_scale", "default", [])]:
        yield ds, var, opts, {}, "k1_class3_and_scale"
    for windows in ("0", "1"):  # the bin table's probe bound and the table-free redo
        for ds, var, opts in [("syn_small", "default", []), ("syn_dna", "default", [])]:
            yield ds, var, opts, {"GHOSTM_K1_PROBE_WINDOWS": windows}, f"k1_probe_windows_{windows}"
    for ds, var, opts in [("syn_small", "default", []), ("syn_dna", "default", [])]:
        yield ds, var, opts, {"GHOSTM_SEGMENT_CANDS": "300", "GHOSTM_TAIL_CANDS": "40"}, "segments"


def main():
    group, root = sys.argv[1], sys.argv[2]
    info = (native.load().GhostmBuildInfo() or b"").decode()
    if "LDS poison build" not in info:
        print(json.dumps({"error": f"not the poison build: {info}"}), flush=True)
        sys.exit(2)
    golden = json.load(open(os.path.join(cases.GOLDEN, "golden.json")))
    runs, failures, forms = 0, [], set()
    for ds, var, opts, env, form in plan(group):
        d = cases.build_dataset(ds, root)
        if env.get("GHOSTM_K1_CAPS") == "@caps":
            env = dict(env, GHOSTM_K1_CAPS=caps(d))
        text, st = run(d, opts, env)
        runs += 1
        forms.add(form)
        want = golden["aln"][f"{ds}/{var}"]["sha256"]
        if hashlib.sha256(text).hexdigest() != want:
            failures.append(f"{ds}/{var} {form}")
        if form.startswith("k1_classes") and not all(st[f"seed_queries_class{c}"] > 0 for c in range(4)):
            failures.append(f"{ds}/{var} {form}: not every K1 class ran")
    print(json.dumps({"group": group, "pattern": os.environ.get("GHOSTM_LDS_POISON_PATTERN"), "runs": runs,
                      "forms": sorted(forms), "failures": failures}), flush=True)
    sys.exit(1 if failures else 0)


if __name__ == "__main__":
    main()
