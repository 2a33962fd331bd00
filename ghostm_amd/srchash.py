"""The source hash of the native library: sha256 over ghostm_amd/csrc's sources
(*.h, *.cpp, *.hip, Makefile) and include/ghostm_hip.h, by file name and content,
first 16 hex digits. The Makefile compiles it into every build
(GhostmBuildInfo: "... src <hash>"); tests/conftest.py refuses a library whose
hash is not the tree's, and bench.py trusts a PMC summary only when it was
recorded on a library with the hash it is timing. No imports beyond the standard
library: the Makefile runs this file as a script.
"""
from __future__ import annotations

import hashlib
import os
import re

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")


def source_files() -> list[str]:
    names = sorted(n for n in os.listdir(CSRC)
                   if n == "Makefile" or n.endswith((".h", ".cpp", ".hip")))
    return [os.path.join(CSRC, n) for n in names] + [os.path.join(REPO_DIR, "include", "ghostm_hip.h")]


def tree_hash() -> str:
    h = hashlib.sha256()
    for p in source_files():
        h.update(os.path.relpath(p, REPO_DIR).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(hashlib.sha256(f.read()).digest())
    return h.hexdigest()[:16]


def info_hash(build_info: str) -> str | None:
    """The hash a library reports in GhostmBuildInfo, or None (older builds)."""
    m = re.search(r"\bsrc ([0-9a-f]{16})\b", build_info or "")
    return m.group(1) if m else None


if __name__ == "__main__":
    print(tree_hash())
