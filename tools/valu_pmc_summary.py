"""Cycles per wave64 VALU instruction from a rocprofv3 PMC pass over the
tools/microbench/valu_issue binary (GRBM_GUI_ACTIVE / 8 XCDs = shader clock
cycles over the dispatch, the same clock pmc_summary.py reports for the bench
kernels), so the microbench and the kernels are priced in the same units.

  rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES \
      --output-format csv -d OUT -o run -- tools/microbench/build/valu_issue
  python tools/valu_pmc_summary.py OUT/run_counter_collection.csv [valu_waves]

With `valu_waves` the names come from tools/microbench/valu_waves.hip (one
opcode, 16 chains per wave, at 1/2/4/8 waves per SIMD).
"""
import collections
import csv
import os
import re
import sys

SIMDS = 256 * 4


def main(path: str, bench: str = "valu_issue") -> None:
    if os.path.isdir(path):  # a rocprofv3 -d directory: its counter collection file
        import glob

        path = sorted(glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True))[0]
    d = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        key = (int(r["Dispatch_Id"]), r["Kernel_Name"])
        d[key][r["Counter_Name"]] = float(r["Counter_Value"])
        d[key]["dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        d[key]["grid"] = int(r["Grid_Size"])
    src = os.path.join(os.path.dirname(os.path.abspath(__file__)), "microbench", bench + ".hip")
    names = {}
    for ln in open(src):
        m = re.match(r'\s*X\((\d+), "([^"]+)"', ln)
        if m:
            names[int(m.group(1))] = m.group(2)
        for m in re.finditer(r'run<(\d+)>\("([^"]+)"', ln):
            names[int(m.group(1))] = m.group(2)
    print(f"{'op':30s} {'waves/SIMD':>10s} {'clk GHz':>8s} {'G inst/s':>9s} {'cyc/inst':>8s}")
    for (disp, kn), c in sorted(d.items()):
        if disp % 2 == 1:  # each op runs twice: warm-up, then the timed launch
            continue
        op = int(re.search(r"k<(\d+)>", kn).group(1))
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        w = c["grid"] // 256 // 256
        print(f"{names[op]:30s} {w:10d} {cyc / c['dur'] / 1e9:8.2f} {c['SQ_INSTS_VALU'] / c['dur'] / 1e9:9.1f} "
              f"{SIMDS * cyc / c['SQ_INSTS_VALU']:8.2f}")


if __name__ == "__main__":
    main(*sys.argv[1:3])
