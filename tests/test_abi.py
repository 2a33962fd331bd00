"""The C-ABI library loads on a CPU-only host and exports every function declared in
include/ghostm_hip.h (no device calls here)."""
import ctypes
import os
import subprocess

import cases
from ghostm_amd import native


def test_library_exports_header_functions(built):
    lib = native.load()
    declared = native.header_functions()
    assert len(declared) >= 22
    for name in declared:
        assert hasattr(lib, name), name
        assert name in native.SIGNATURES, f"{name} has no ctypes signature"


def test_reference_plugin_surface_present(built):
    """The ten symbols the reference's aligner.cpp binds (aligner_gpu.h:33-114)."""
    ref = ["InitGpu", "GetNeededGPUMemorySize", "CheckGpuMemory", "SetOptionGpu", "printGpuInfo",
           "SetQueryGpu", "SetDbGpu", "SearchNextGpu", "CalculateScoreGpu", "FreeGpu"]
    out = subprocess.run(["nm", "-D", "--defined-only", native.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    for s in ref:
        assert s in exported, s


def test_hit_record_layout():
    assert ctypes.sizeof(native.GhostmHit) == 32
    from ghostm_amd.aligner import HIT_DTYPE

    assert HIT_DTYPE.itemsize == 32


def test_reference_host_links_against_plugin():
    """Where the reference was compiled here, ghostm_ref_plugin resolves the ten
    plugin symbols from libghostm_hip.so (drop-in at the symbol level), while the
    oracle build ghostm_ref does not link the product at all."""
    if not os.path.exists(cases.REF_PLUGIN):
        import pytest

        pytest.skip("oracle/_ref not built (no /root/reference here)")
    out = subprocess.run(["ldd", cases.REF_PLUGIN], capture_output=True, text=True, check=True).stdout
    assert "libghostm_hip.so" in out
    und = subprocess.run(["nm", "-D", "--undefined-only", cases.REF_PLUGIN], capture_output=True,
                         text=True, check=True).stdout
    for s in ["SearchNextGpu", "CalculateScoreGpu", "SetDbGpu", "SetQueryGpu"]:
        assert s in und
    out = subprocess.run(["ldd", cases.REF], capture_output=True, text=True, check=True).stdout
    assert "libghostm_hip.so" not in out and "libamdhip64" not in out


def test_reference_oracle_traps_gpu_path(tmp_path):
    """The oracle build's GPU symbols are the exit(2) trap stub (oracle/gpu_trap.c):
    asking it for -D fails loudly instead of running anything."""
    if not os.path.exists(cases.REF):
        import pytest

        pytest.skip("oracle/_ref not built (no /root/reference here)")
    d = tmp_path
    subprocess.run([cases.GHOSTM, "qry", "-i", os.path.join(cases.GOLDEN, "testset_queries.fasta"),
                    "-o", str(d / "q")], check=True, capture_output=True)
    subprocess.run([cases.GHOSTM, "db", "-i", os.path.join(cases.GOLDEN, "testset_db.fasta"),
                    "-o", str(d / "db")], check=True, capture_output=True)
    r = subprocess.run([cases.REF, "aln", "-i", str(d / "q"), "-d", str(d / "db"), "-o", str(d / "o"),
                        "-D", "0"], capture_output=True)
    assert r.returncode == 2 and b"called in the CPU oracle build" in r.stderr


def test_cli_usage_and_unknown_command(built):
    r = subprocess.run([cases.GHOSTM], capture_output=True)
    assert r.returncode == 1
    r = subprocess.run([cases.GHOSTM, "nope"], capture_output=True)
    assert r.returncode == 1 and b"unrecognized command" in r.stderr


def test_unsupported_score_option_exits_zero(tmp_path, built):
    """statistics.cpp:143-145 + main.cpp:116-121: -y 0 with an unknown matrix/gap
    combination prints the error, writes nothing, exits 0 (no device touched)."""
    r = subprocess.run([cases.GHOSTM, "aln", "-i", "x", "-d", "y", "-o", str(tmp_path / "o"),
                        "-G", "5"], capture_output=True)
    assert r.returncode == 0
    assert b"not support score option" in r.stderr
    assert not (tmp_path / "o").exists()


def test_library_source_hash_matches_tree(built):
    """The built libraries report the source hash of this tree (GhostmBuildInfo
    "src <hash>", ghostm_amd/srchash.py), and ghostm_amd/lib holds only the two
    product libraries: the GPU suite refuses to run otherwise (conftest.py)."""
    from conftest import library_hash_mismatch

    assert library_hash_mismatch() is None


def test_source_hash_covers_the_native_sources(tmp_path):
    """ghostm_amd/srchash.py hashes every csrc source and the header by name and
    content (the Makefile compiles the same hash into GhostmBuildInfo), and
    info_hash reads it back from a build-info string."""
    from ghostm_amd import srchash

    files = [os.path.relpath(p, srchash.REPO_DIR) for p in srchash.source_files()]
    assert "include/ghostm_hip.h" in files
    for name in ("kernels.h", "device.hip", "aligner.cpp", "Makefile"):
        assert os.path.join("ghostm_amd", "csrc", name) in files
    h = srchash.tree_hash()
    assert len(h) == 16 and int(h, 16) >= 0
    assert srchash.info_hash(f"ghostm_hip gfx950: K1 ...; LDS poison build; src {h}") == h
    assert srchash.info_hash("ghostm_hip gfx950: K1 ...") is None
