"""K1 phase 0's entry -> list byte table (ghostm_amd/csrc/seed_lists.h, shared
with k_seed_filter): compiled with g++ and checked against a per-entry walk over
the list offsets on random list sets (empty lists, boundaries at every position
of a 16-entry window). The kernel itself runs in the GPU parity tests."""
import os
import subprocess


def test_seed_list_bytes(tmp_path):
    src = os.path.join(os.path.dirname(__file__), "native", "test_seed_lists.cpp")
    exe = str(tmp_path / "test_seed_lists")
    subprocess.run(["g++", "-O2", "-std=c++17", src, "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "trials ok" in r.stdout
