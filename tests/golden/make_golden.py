"""Regenerate tests/golden/golden.json and the small full-text fixtures.

Runs ONLY in the build container, where the reference CPU program oracle/_ref/
ghostm_ref is compiled from /root/reference (see oracle/Makefile). For every dataset
of tests/cases.py it formats the inputs with the REFERENCE formatters and records
the sha256 of every formatted file; then it runs the reference `aln` for every
variant and records sha256 + line count of the output. Small outputs are also kept
as text (readme_kat.out, protein_*.out).

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import shutil
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cases  # noqa: E402


def ref_dataset(name: str, root: str) -> str:
    """Same inputs as cases.build_dataset, but formatted by the reference program."""
    d = os.path.join(root, name)
    os.makedirs(d, exist_ok=True)
    for tool, args in cases.DATASETS[name]:
        a = [x.format(d=d, golden=cases.GOLDEN) for x in args]
        if tool == "py":  # deterministic data generation (cases.py), no reference code
            getattr(cases, a[0])(*a[1:])
            continue
        exe = cases.GHOSTM if tool == "synth" else cases.REF
        subprocess.run([exe, tool] + a, check=True, capture_output=True)
    return d


def main() -> None:
    if not os.path.exists(cases.REF):
        raise SystemExit("oracle/_ref/ghostm_ref missing: make -C oracle ref")
    out = {"formatted": {}, "aln": {}, "generator": "tests/golden/make_golden.py",
           "reference": "oracle/_ref/ghostm_ref (reference CPU path, g++ -O2)"}
    tmp = tempfile.mkdtemp(prefix="ghostm_golden_")
    try:
        for name in cases.DATASETS:
            d = ref_dataset(name, tmp)
            out["formatted"][name] = {f: cases.sha256(os.path.join(d, f)) for f in cases.formatted_files(d)}
        for ds, var, opts, env in cases.VARIANTS:
            d = os.path.join(tmp, ds)
            path = os.path.join(tmp, f"{ds}.{var}.out")
            text = cases.run_aln(cases.REF, d, opts, env, path)
            out["aln"][f"{ds}/{var}"] = {"sha256": cases.sha256(path), "lines": text.count(b"\n"),
                                         "bytes": len(text)}
            if ds == "readme_kat" and var == "default":
                shutil.copy(path, os.path.join(cases.GOLDEN, "readme_kat.out"))
            if ds == "protein_testset":
                shutil.copy(path, os.path.join(cases.GOLDEN, f"protein_{var}.out"))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    with open(os.path.join(cases.GOLDEN, "golden.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", os.path.join(cases.GOLDEN, "golden.json"))


if __name__ == "__main__":
    main()
