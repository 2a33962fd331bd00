"""Run one golden dataset/option variant N times through the HIP path in one
process and report, for every run whose text differs from the CPU oracle's,
which lines differ (diagnosing a nondeterministic result).

    python tools/repeat_variant.py syn_small "-b 20 -t 1 -y 2" 20
"""
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import cases  # noqa: E402
from ghostm_amd.aligner import Session  # noqa: E402


def main():
    ds, opts, n = sys.argv[1], sys.argv[2].split(), int(sys.argv[3])
    root = tempfile.mkdtemp()
    d = cases.build_dataset(ds, root)
    want_path = os.path.join(root, "oracle.out")
    subprocess.run([cases.ORACLE, "aln", "-i", d + "/q", "-d", d + "/db", "-o", want_path] + opts, check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    want = open(want_path, "rb").read().split(b"\n")
    bad = 0
    for r in range(n):
        with Session(["-i", d + "/q", "-d", d + "/db", "-o", os.devnull, "-D", "0"] + opts) as s:
            s.run()
            got = s.output().split(b"\n")
        diff = [(i, a, b) for i, (a, b) in enumerate(zip(got, want)) if a != b]
        if diff or len(got) != len(want):
            bad += 1
            print(f"run {r}: {len(diff)} lines differ (lines {len(got)} vs {len(want)})", flush=True)
            for i, a, b in diff[:6]:
                print(f"  line {i}\n    gpu    {a.decode()}\n    oracle {b.decode()}", flush=True)
    print(f"{bad} of {n} runs differ", flush=True)


if __name__ == "__main__":
    main()
