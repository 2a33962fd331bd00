"""Summarise a tools/profile.sh run into profiles/ (tracked):

  profiles/<round>_kernel_stats.csv   rocprofv3 --stats of the bench command
  profiles/<round>_pmc.json           per kernel: launches, mean duration, HBM bytes
                                      per launch (FETCH_SIZE x 2 x 1024 on gfx950, see
                                      MI355X_MICROARCH.md §HBM; WRITE_SIZE x 1024), SQ
                                      issue counters and the VALU issue utilisation
  profiles/pmc_traffic.json           the per-launch HBM bytes bench.py reports as
                                      roofline.traffic
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
import shutil
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIMDS = 256 * 4


def short(name: str) -> str:
    n = re.sub(r"^void\s+", "", name)
    n = n.split("(")[0]
    return n.replace("ghostm::kern::", "")


def rows(pattern: str):
    for path in glob.glob(pattern, recursive=True):
        with open(path, newline="") as f:
            yield from csv.DictReader(f)


def counters(d: str) -> dict:
    """kernel -> counter -> list of per-dispatch values; kernel -> durations (ns)."""
    vals: dict = defaultdict(lambda: defaultdict(dict))
    dur: dict = defaultdict(dict)
    for r in rows(os.path.join(d, "**", "*counter_collection.csv")):
        k = short(r["Kernel_Name"])
        disp = r.get("Dispatch_Id") or r.get("Correlation_Id")
        vals[k][r["Counter_Name"]][disp] = vals[k][r["Counter_Name"]].get(disp, 0.0) + float(r["Counter_Value"])
        if r.get("Start_Timestamp") and r.get("End_Timestamp"):
            dur[k][disp] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return vals, dur


def library_hash() -> dict:
    """The profiled library's GhostmBuildInfo and source hash (ghostm_amd/srchash.py):
    bench.py uses these counters only while it times a library with the same hash."""
    import ctypes
    import sys

    sys.path.insert(0, REPO)
    from ghostm_amd import native, srchash

    lib = ctypes.CDLL(native.LIB_PATH)
    lib.GhostmBuildInfo.restype = ctypes.c_char_p
    info = lib.GhostmBuildInfo().decode()
    return {"library": os.path.relpath(native.LIB_PATH, REPO), "library_build_info": info,
            "library_src_hash": srchash.info_hash(info), "tree_src_hash": srchash.tree_hash()}


def mean(xs):
    xs = list(xs)
    return sum(xs) / len(xs) if xs else None


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", required=True)
    ap.add_argument("--prof", required=True)
    ap.add_argument("--queries", type=int, required=True)
    ap.add_argument("--preset", default="cfg4", help="bench preset profiled (pmc_traffic_<preset>.json)")
    ap.add_argument("--trace-runs", type=int, default=3, help="session runs in the traced command (warmup + steps)")
    args = ap.parse_args()
    prof = os.path.join(REPO, "profiles")
    os.makedirs(prof, exist_ok=True)

    stats = glob.glob(os.path.join(args.prof, "trace", "**", "*kernel_stats.csv"), recursive=True)
    kernels: dict = {}
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{args.round}_kernel_stats.csv"))
        for r in rows(stats[0]):
            kernels[short(r["Name"])] = {"launches_in_trace": int(r["Calls"]),
                                         "avg_ms_trace": float(r["AverageNs"]) / 1e6,
                                         "percent_of_gpu_time": float(r["Percentage"])}

    fetch, _ = counters(os.path.join(args.prof, "fetch"))
    write, _ = counters(os.path.join(args.prof, "write"))
    sq, sq_dur = counters(os.path.join(args.prof, "sq"))
    lds, _ = counters(os.path.join(args.prof, "lds"))
    issue = {}
    ipath = os.path.join(prof, "r2_valu_issue.json")
    if os.path.exists(ipath):
        with open(ipath) as f:
            issue = json.load(f)
    for k in set(fetch) | set(write) | set(sq) | set(lds):
        e = kernels.setdefault(k, {})
        f = mean(fetch.get(k, {}).get("FETCH_SIZE", {}).values())
        w = mean(write.get(k, {}).get("WRITE_SIZE", {}).values())
        if f is not None:
            e["fetch_size_kb_raw"] = f
            e["hbm_read_bytes_per_launch"] = f * 1024 * 2  # gfx950: FETCH_SIZE reads 1/2
        if w is not None:
            e["hbm_write_bytes_per_launch"] = w * 1024
        if f is not None and w is not None:
            e["hbm_bytes_per_launch"] = e["hbm_read_bytes_per_launch"] + e["hbm_write_bytes_per_launch"]
        if k in sq:
            c = {name: mean(v.values()) for name, v in sq[k].items()}
            e["sq"] = c
            d = mean(sq_dur.get(k, {}).values())
            if d:
                e["avg_ms_pmc_pass"] = d / 1e6
            # a wave64 VALU instruction occupies its SIMD for 2 cycles; the clock is
            # GRBM_GUI_ACTIVE / 8 XCDs over the dispatch (MI355X_MICROARCH.md, DVFS)
            if c.get("SQ_INSTS_VALU") and c.get("GRBM_GUI_ACTIVE"):
                cyc = c["GRBM_GUI_ACTIVE"] / 8
                e["valu_issue_util"] = c["SQ_INSTS_VALU"] * 2 / (SIMDS * cyc)
                e["valu_insts_per_launch"] = c["SQ_INSTS_VALU"]
                if d:
                    e["effective_clock_ghz"] = cyc / d
                    # against the measured chip-wide issue rate of packed/VOP3 ops
                    if issue.get("packed_vop3_ginst_s"):
                        e["valu_frac_of_measured_issue"] = c["SQ_INSTS_VALU"] / d / issue["packed_vop3_ginst_s"]
        if k in lds:
            c = {name: mean(v.values()) for name, v in lds[k].items()}
            e["lds"] = c
            if c.get("SQ_LDS_IDX_ACTIVE") and c.get("SQ_LDS_BANK_CONFLICT") is not None:
                busy = c["SQ_LDS_IDX_ACTIVE"] - c["SQ_LDS_BANK_CONFLICT"]
                e["lds_bank_conflict_rate"] = c["SQ_LDS_BANK_CONFLICT"] / busy if busy > 0 else None
    lib = library_hash()
    with open(os.path.join(prof, f"{args.round}_pmc.json"), "w") as f:
        json.dump({"round": args.round, "queries": args.queries, "preset": args.preset, **lib, "kernels": kernels},
                  f, indent=1, sort_keys=True)

    def fam(prefix):
        best = [k for k in kernels if k.startswith(prefix) and "hbm_bytes_per_launch" in kernels[k]]
        if not best:
            return None
        k = max(best, key=lambda x: kernels[x].get("percent_of_gpu_time", 0))
        return kernels[k]["hbm_bytes_per_launch"]

    # K1 = every seed-stage kernel; per bench step = bytes per launch x launches
    # in the trace / runs in the trace (warmup + steps of the traced command)
    k1 = [k for k in kernels if k.startswith(("k_seed", "k_compact")) and "hbm_bytes_per_launch" in kernels[k]]
    k1_step = sum(kernels[k]["hbm_bytes_per_launch"] * kernels[k].get("launches_in_trace", 0) for k in k1)
    k1v = [k for k in kernels if k.startswith(("k_seed", "k_compact")) and "valu_insts_per_launch" in kernels[k]]
    k1v_step = sum(kernels[k]["valu_insts_per_launch"] * kernels[k].get("launches_in_trace", 0) for k in k1v)
    k2 = [k for k in kernels if k.startswith("k_score") and "valu_insts_per_launch" in kernels[k]]
    k2_main = max(k2, key=lambda x: kernels[x].get("percent_of_gpu_time", 0)) if k2 else None
    traffic = {"round": args.round, "queries": args.queries, "preset": args.preset, **lib,
               "note": "HBM bytes per launch = FETCH_SIZE*2*1024 + WRITE_SIZE*1024 (gfx950 correction); "
                       "VALU instructions = SQ_INSTS_VALU per dispatch",
               "k_score_hbm_bytes_per_launch": fam("k_score"),
               "k_score_valu_insts_per_launch": kernels[k2_main]["valu_insts_per_launch"] if k2_main else None,
               # shader cycles per wave64 VALU instruction on one SIMD (GRBM_GUI_ACTIVE / 8 XCDs
               # over the dispatch, 1024 SIMDs), the unit of profiles/r2c_valu_issue_pmc.txt
               "k_score_valu_cycles_per_inst": (2.0 / kernels[k2_main]["valu_issue_util"])
               if k2_main and kernels[k2_main].get("valu_issue_util") else None,
               "k_score_effective_clock_ghz": kernels[k2_main].get("effective_clock_ghz") if k2_main else None,
               "k1_hbm_bytes_per_step": k1_step / args.trace_runs if k1 else None,
               "k1_valu_insts_per_step": k1v_step / args.trace_runs if k1v else None,
               "k1_kernels": sorted(k1)}
    names = [f"pmc_traffic_{args.preset}.json"] + (["pmc_traffic.json"] if args.preset == "cfg4" else [])
    for name in names:
        with open(os.path.join(prof, name), "w") as f:
            json.dump(traffic, f, indent=1)
    print(json.dumps(traffic))


if __name__ == "__main__":
    main()
